"""Multi-rank render check, launched by tests/test_gpu_parity.py under torchrun.

Every rank renders its row band (nerf_amd.distributed.band); the bands are
all-gathered, and, separately, rendered as packed tiles and gathered to rank 0.
Rank 0 compares both frames with a single-call full-frame render (bit-identical
expected: rays are independent) and prints one JSON line.
Backend from NERF_DIST_BACKEND (the two-rank test uses gloo so that two ranks can
share one device; the 8-GPU bench uses RCCL).  With NERF_DIST_FORCE_GROUP=1 and one
rank the same code runs over an RCCL process group of world size 1 (the one-GPU
box's check of the nccl branches), plus an RCCL all-reduce of a gradient-store-
sized device tensor.  Every rank prints one JSON line.
"""
import json
import os
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "nerf-dbr_amd")]


def main():
    import torch
    import torch.distributed as dist

    from nerf_amd import distributed as D
    from nerf_amd import weights as W
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    rank, world, _, dev = D.init_from_env()
    ckpt = W.write_synthetic_checkpoint(os.path.join(tempfile.mkdtemp(), "ckpt.pth"), seed=0)
    r = MI355XRenderer(os.environ.get("NERF_CHECK_PRECISION", "bf16"), device_index=dev)
    r.setup(ckpt)
    pose = torch.eye(4)
    pose[2, 3] = 4.0
    w, h, s = 96, 37, 32                       # 37 rows: uneven bands
    rgb, depth = D.render_sharded(r.render_rows, pose, (w, h), s)          # all-gather of the bands
    root = D.render_frame_to_root(r, pose, (w, h), s)                    # packed tiles gathered to rank 0
    ok = None
    if rank == 0:
        ref_rgb, ref_depth = r.render_image(pose, (w, h), s)
        ok = bool(torch.equal(rgb, ref_rgb) and torch.equal(depth, ref_depth)
                  and torch.equal(root[0], ref_rgb) and torch.equal(root[1], ref_depth))
    else:
        ok = root is None
    rec = {"world": world, "rank": rank, "backend": dist.get_backend(), "bands": D.bands(world, h), "identical": ok}
    if dist.get_backend() == "nccl":
        # the training step's exchange: one all-reduce (SUM) of the 2 x 530,052-float gradient store
        g = torch.arange(2 * 530_052, dtype=torch.float32, device="cuda") * (rank + 1)
        dist.all_reduce(g)
        want = torch.arange(2 * 530_052, dtype=torch.float32, device="cuda") * (world * (world + 1) // 2)
        rec["all_reduce_ok"] = bool(torch.equal(g, want))
        rec["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
        ok = ok and rec["all_reduce_ok"]
    print(json.dumps(rec), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
