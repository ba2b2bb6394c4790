import os, sys, tempfile
import torch
sys.path[:0] = ['.', 'nerf-dbr_amd']
from nerf_amd import weights as W
from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer
import bench
ck = W.write_lego_checkpoint(os.path.join(tempfile.mkdtemp(), 'l.pth'))
pose = torch.eye(4); pose[2, 3] = 4.0
r32 = MI355XRenderer("fp32"); r32.setup(ck); r32.hip.set_profiling(True)
out, f8 = bench.other_configs(ck, pose, 0, r32)
g = out["gate_path_f16x3_800x600x128"]
print("other_configs", g["rgb_max_abs_vs_fp32_band"], g["depth_max_abs_vs_fp32_band"])
x3 = MI355XRenderer("f16x3"); x3.setup(ck)
a, da = x3.render_rows(pose, (800, 600), 128, 292, 308); b, db = r32.render_rows(pose, (800, 600), 128, 292, 308)
print("after", float((a - b).abs().max()), x3.hip is r32.hip, x3.precision)
