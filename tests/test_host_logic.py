"""CPU tests of the host-side logic: checkpoints, the plugin interface, the suite's
CSV/rays-per-second contract and the multi-process band gather (gloo, world size 2)."""
import os

import numpy as np
import pytest
import torch

from nerf_amd import distributed as D
from nerf_amd import weights as W
from nerf_amd.benchmark import base_renderer as B
from nerf_amd.benchmark.benchmark_suite import CSV_COLUMNS, UnifiedBenchmarkSuite, generate_test_poses


def test_param_counts():
    assert W.N_PARAMS == 530052
    assert W.FLOPS_PER_SAMPLE == 1055744


def test_checkpoint_roundtrip(tmp_path):
    c, f = W.synthetic_models(5)
    p = W.save_checkpoint(str(tmp_path / "ck.pth"), c, f)
    c2, f2 = W.load_checkpoint(p)
    assert W.state_dict_digest(c) == W.state_dict_digest(c2)
    assert W.state_dict_digest(f) == W.state_dict_digest(f2)


def test_checkpoint_reference_layout_with_extra_keys(tmp_path):
    """Trainer checkpoints carry optimizer/config entries too (trainer.py:376-384)."""
    c, f = W.synthetic_models(1)
    ck = {"coarse_model": {k: torch.from_numpy(v) for k, v in c.items()},
          "fine_model": {k: torch.from_numpy(v) for k, v in f.items()},
          "config": {"lr": 5e-4, "n_samples": 64}, "train_losses": [0.1, 0.05], "val_losses": []}
    p = str(tmp_path / "trainer.pth")
    torch.save(ck, p)
    c2, f2 = W.load_checkpoint(p)
    assert W.state_dict_digest(f) == W.state_dict_digest(f2)


@pytest.mark.parametrize("legacy_numpy_names", [False, True])
def test_checkpoint_with_numpy_float64_losses(tmp_path, legacy_numpy_names):
    """The reference trainer's loss histories are np.float64 (np.mean, trainer.py:336-345);
    the weights-only loader admits them, also under the numpy<2 module path."""
    import zipfile

    c, f = W.synthetic_models(2)
    ck = {"coarse_model": {k: torch.from_numpy(v) for k, v in c.items()},
          "fine_model": {k: torch.from_numpy(v) for k, v in f.items()},
          "train_losses": [np.mean([0.1, 0.2]), np.mean([0.05])], "val_losses": [np.float64(0.3)]}
    p = str(tmp_path / "ref_trainer.pth")
    torch.save(ck, p)
    if legacy_numpy_names:
        q = str(tmp_path / "ref_trainer_legacy.pth")
        with zipfile.ZipFile(p) as zin, zipfile.ZipFile(q, "w", compression=zipfile.ZIP_STORED) as zout:
            for it in zin.infolist():
                data = zin.read(it.filename)
                if it.filename.endswith("data.pkl"):
                    assert b"numpy._core.multiarray" in data
                    data = data.replace(b"numpy._core.multiarray", b"numpy.core.multiarray")
                zout.writestr(it, data)
        p = q
    with pytest.raises(Exception):
        torch.load(p, weights_only=True)            # what the plain weights-only load does
    c2, f2 = W.load_checkpoint(p)
    assert W.state_dict_digest(f) == W.state_dict_digest(f2)
    raw = W.torch_load_weights_only(p)
    assert [float(v) for v in raw["train_losses"]] == [0.15000000000000002, 0.05]


def test_blender_loader_contract(tmp_path):
    """nerf_amd.data follows src/data/loader.py:13-129: RGBA -> Lanczos resize -> /255 ->
    white composite, focal from camera_angle_x, missing split skipped with a warning."""
    from PIL import Image

    from blender_fixture import write_blender_dataset
    from nerf_amd.data import load_synthetic_data

    raw = write_blender_dataset(str(tmp_path), splits=(("train", 2), ("test", 1)), size=(12, 10))
    ds = load_synthetic_data(str(tmp_path), img_wh=(24, 20))
    assert set(ds) == {"train", "test"}
    tr = ds["train"]
    assert len(tr) == 2 and np.isclose(tr.focal, 0.5 * 24 / np.tan(0.5 * 0.6911112070083618))
    a = np.array(Image.fromarray(raw["train"][1], "RGBA").resize((24, 20), Image.LANCZOS)) / 255.0
    want = a[..., :3] * a[..., 3:4] + (1 - a[..., 3:4])
    item = tr[1]
    assert item["image"].shape == (20, 24, 3) and item["pose"].shape == (4, 4)
    assert np.allclose(item["image"].numpy(), want.astype(np.float32))


def test_cli_refuses_to_overwrite_a_trained_model(tmp_path):
    import main as cli

    with pytest.raises(SystemExit):
        cli.main(["--synthetic-checkpoint", "--checkpoint", str(tmp_path / "ck.pth")])
    assert not os.path.exists(tmp_path / "ck.pth")


def test_strict_state_dict():
    sd = W.synthetic_state_dict(0)
    del sd["density_head.bias"]
    with pytest.raises(KeyError):
        W.validate_state_dict(sd)


def test_shared_model_missing_checkpoint_falls_back(tmp_path, capsys):
    B.SharedNeRFModel.reset()
    m = B.SharedNeRFModel()
    m.load_models(str(tmp_path / "nope.pth"), "cuda")
    coarse, fine = m.get_models("cuda")
    assert "randomly initialized" in capsys.readouterr().out
    W.validate_state_dict(coarse)
    B.SharedNeRFModel.reset()


def test_mi355x_renderer_fails_loudly_without_gpu():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    with pytest.raises(RuntimeError):
        MI355XRenderer("bf16")


def test_poses_match_reference_fixture(golden):
    g = golden("rays")
    poses = generate_test_poses(2)
    for i in range(2):
        assert np.array_equal(poses[i].numpy(), g["poses"][i])


class FakeRenderer(B.BaseUnifiedRenderer):
    """CPU stand-in that only exercises the suite's plumbing."""

    def __init__(self):
        super().__init__("Fake", "cpu")

    def render_image(self, camera_pose, resolution, samples_per_ray=64):
        w, h = resolution
        return torch.full((h, w, 3), 0.5), torch.full((h, w), 3.0)

    def execute_volume_rendering(self, densities, colors, z_vals, ray_directions):
        raise NotImplementedError

    def query_nerf_networks(self, positions, directions, use_fine=True):
        raise NotImplementedError

    def generate_rays(self, camera_pose, width, height, focal=800.0):
        raise NotImplementedError

    def sample_points_on_rays(self, rays_o, rays_d, n_samples=64):
        raise NotImplementedError


def test_suite_csv_contract(tmp_path):
    ck = W.write_synthetic_checkpoint(str(tmp_path / "ck.pth"))
    suite = UnifiedBenchmarkSuite(str(tmp_path / "out"), warmup=0)
    suite.renderers.append(FakeRenderer())
    suite.run_benchmark(ck, [(20, 10)], [8], n_views=2)
    df = suite.generate_report(plot=False)
    assert list(df.columns) == CSV_COLUMNS
    row = df.iloc[0]
    assert row["Resolution"] == "20x10" and row["Samples/Ray"] == 8
    assert np.isclose(row["Rays/Second"], 200 / row["Render Time (s)"])
    assert os.path.exists(tmp_path / "out" / "benchmark_results.csv")
    assert os.path.exists(tmp_path / "out" / "sample_renders" / "Fake" / "view_1_rgb.png")


@pytest.mark.parametrize("world,height", [(1, 600), (2, 600), (8, 600), (8, 150), (3, 7), (4, 2)])
def test_bands_partition_rows(world, height):
    b = D.bands(world, height)
    assert b[0][0] == 0 and b[-1][1] == height
    assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
    assert max(r1 - r0 for r0, r1 in b) - min(r1 - r0 for r0, r1 in b) <= 1


def _gather_worker(rank, world, port, width, height, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def render_rows(pose, res, spp, r0, r1):
        rows = torch.arange(r0, r1, dtype=torch.float32)[:, None].expand(r1 - r0, width)
        cols = torch.arange(width, dtype=torch.float32)[None, :].expand(r1 - r0, width)
        rgb = torch.stack([rows, cols, rows * 1000 + cols], -1)
        return rgb, rows + 0.5

    rgb, depth = D.render_sharded(render_rows, None, (width, height), 4)

    class Tiler:                  # the renderer surface render_frame_to_root uses
        def torch_device(self):
            return torch.device("cpu")

        def render_band(self, pose, res, spp, r0, r1, out):
            c, d = render_rows(pose, res, spp, r0, r1)
            out[: r1 - r0, :, :3] = c
            out[: r1 - r0, :, 3] = d
            return out

    first = D.render_frame_to_root(Tiler(), None, (width, height), 4)
    kept = None if first is None else (first[0].clone(), first[1].clone())

    class Tiler2(Tiler):          # a second, different frame
        def render_band(self, pose, res, spp, r0, r1, out):
            super().render_band(pose, res, spp, r0, r1, out)
            out[: r1 - r0] *= -1.0
            return out

    second = D.render_frame_to_root(Tiler2(), None, (width, height), 4)
    if first is not None:
        # the first frame the caller kept is not overwritten by the next gather
        assert torch.equal(first[0], kept[0]) and torch.equal(first[1], kept[1])
        assert torch.equal(second[0], -kept[0]) and torch.equal(second[1], -kept[1])
    root = None if first is None else (first[0].contiguous().numpy(), first[1].contiguous().numpy())
    q.put((rank, rgb.numpy(), depth.numpy(), root))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("height", [10, 7])
def test_band_gather_gloo_world2(height):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    width = 5
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, width, height, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    rows = np.arange(height, dtype=np.float32)[:, None].repeat(width, 1)
    cols = np.arange(width, dtype=np.float32)[None, :].repeat(height, 0)
    for rank, rgb, depth, root in outs:
        assert np.array_equal(rgb, np.stack([rows, cols, rows * 1000 + cols], -1))
        assert np.array_equal(depth, rows + 0.5)
        # gather of the packed band tiles to rank 0 only
        if rank == 0:
            assert np.array_equal(root[0], rgb) and np.array_equal(root[1], depth)
        else:
            assert root is None


class _FakeTrainer:
    """A linear stand-in for MI355XTrainer: a share's 'gradient' is sum over its rays of
    g(ray) / n_total, so the all-reduced sum must equal the single-rank full step."""

    def __init__(self):
        import torch

        self.g = torch.zeros(6, dtype=torch.float64)
        self.loss = torch.zeros(3, dtype=torch.float64)
        self.updates = 0

    def grad_tensor(self):
        return self.g

    def backward(self, batch, select, t_rand, n_rays_total):
        import torch

        feat = torch.stack([select.double(), t_rand.double().sum(1), select.double() ** 2,
                            torch.ones_like(select.double()), t_rand.double()[:, 0], select.double() % 7], 1)
        self.g.copy_(feat.sum(0) / n_rays_total)
        self.loss.copy_(torch.tensor([1.0, 2.0, 3.0], dtype=torch.float64) * select.numel() / n_rays_total)
        return self.loss

    def update(self):
        self.updates += 1


def _train_worker(rank, world, port, n, q):
    import torch
    import torch.distributed as dist

    from nerf_amd import distributed as D

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    gen = torch.Generator().manual_seed(11)        # the same step draw on every rank
    select = torch.randperm(4096, generator=gen)[:n]
    t_rand = torch.rand(n, 4, generator=gen)
    tr = _FakeTrainer()
    loss = D.train_step_sharded(tr, None, select, t_rand)
    full = _FakeTrainer()
    full.backward(None, select, t_rand, n)
    q.put((rank, tr.g.numpy().copy(), loss.numpy().copy(), full.g.numpy().copy(), tr.updates))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n", [37, 2048])
def test_train_step_sharded_gloo_world2(n):
    """Data-parallel training step: shares, loss normalisation and the gradient all-reduce."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_train_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    for rank, g, loss, full, updates in outs:
        assert np.allclose(g, full, rtol=1e-12, atol=0), rank      # reduced share sums == the full step
        assert np.allclose(loss, [1.0, 2.0, 3.0], rtol=1e-12), rank
        assert updates == 1


# ---------------------------------------- plugin interface vs the reference --
def _sig_fixture():
    import json

    with open(os.path.join(os.path.dirname(__file__), "golden", "plugin_signatures.json")) as f:
        return json.load(f)


def _check_conforms(cls, ref_methods, skip=()):
    import inspect

    for name, spec in ref_methods.items():
        if name in skip:
            continue
        assert hasattr(cls, name), f"{cls.__name__} lacks {name}"
        ours = list(inspect.signature(getattr(cls, name)).parameters.values())
        ref = spec["params"]
        # the reference's parameters, in order and with the same defaults, then
        # only optional extras
        assert [p.name for p in ours[: len(ref)]] == [p["name"] for p in ref], (cls.__name__, name)
        for p, rp in zip(ours, ref):
            if rp["default"] is not None:
                assert p.default is not inspect.Parameter.empty and repr(p.default) == rp["default"], (name, p.name)
        for p in ours[len(ref):]:
            assert p.default is not inspect.Parameter.empty or p.kind == p.VAR_KEYWORD, (name, p.name)


def test_plugin_signatures_match_reference():
    """MI355XRenderer and the restated base class against the reference's
    BaseUnifiedRenderer / SharedNeRFModel signatures (tests/golden/plugin_signatures.json,
    generated from /root/reference/src/benchmark/base_renderer.py:16-281)."""
    import inspect

    from nerf_amd.benchmark.mi355x_renderer import MI355XRenderer

    fx = _sig_fixture()
    _check_conforms(B.BaseUnifiedRenderer, fx["BaseUnifiedRenderer"])
    _check_conforms(B.SharedNeRFModel, fx["SharedNeRFModel"])
    # the plugin: every method (its constructor takes only optional arguments, as
    # the reference's concrete renderers do, so the suite can build it bare)
    _check_conforms(MI355XRenderer, fx["BaseUnifiedRenderer"], skip=("__init__",))
    init = inspect.signature(MI355XRenderer.__init__).parameters
    assert all(p.default is not inspect.Parameter.empty for n, p in init.items() if n != "self")
    # the abstract methods are implemented
    for name, spec in fx["BaseUnifiedRenderer"].items():
        if spec["abstract"]:
            assert not getattr(getattr(MI355XRenderer, name), "__isabstractmethod__", False), name

    class Probe(B.BaseUnifiedRenderer):
        def execute_volume_rendering(self, *a):
            pass

        def render_image(self, *a):
            pass

    probe = Probe("probe", "cpu")
    assert set(fx["BaseUnifiedRenderer.__init__.attributes"]) <= set(vars(probe))
    for k, v in fx["BaseUnifiedRenderer.__init__.values"].items():
        assert repr(getattr(probe, k)) == v, k


def test_bench_self_launch_prints_one_line_world2():
    """`python bench.py --gpus 2` started plainly (no torchrun environment, as a driver may
    start it): bench.py launches torch.distributed.run --nproc-per-node 2 as a child process
    and relays exactly one JSON line, from rank 0, with n_gpus 2 (gloo, no GPU work)."""
    import json
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT", "NERF_BENCH_SELF_LAUNCHED")}
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--launch-check", "--cpu-seconds", "0"], capture_output=True, text=True, timeout=180, env=env,
                       cwd=repo)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["launch_check"] and line["launched_by"] == "self"
    assert line["steps"] == 3 and line["warmup"] == 1


def test_bench_world2_line_carries_cpu_baseline_and_traffic():
    """at N = 2 (gloo, torchrun, no GPU work) rank 0's line carries a
    cpu_baseline, run while rank 1 waits on the TCPStore, and the band-scaled roofline traffic,
    labelled as scaled from the N = 1 counters (half the frame's rays on rank 0's band)."""
    import json
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT", "NERF_BENCH_SELF_LAUNCHED")}
    p = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--launch-check",
                        "--cpu-seconds", "2"], capture_output=True, text=True, timeout=300, env=env, cwd=repo)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    cpu = line["cpu_baseline"]
    assert cpu["unit"] == "rays/s" and cpu["value"] > 0 and cpu["cores"] >= 1 and cpu["kind"] == "port"
    assert "rank 0 of 2" in cpu["n_gpus_protocol"]
    pmc = json.load(open(os.path.join(repo, "profiles", "pmc_latest.json")))["kernels"]["mlp_bf16_kernel"]
    roof = line["roofline"]
    assert roof["kernel"] == "mlp_bf16_kernel"
    assert abs(roof["traffic"] - pmc["hbm_bytes_per_launch"] / 2) < 1e-6 * pmc["hbm_bytes_per_launch"]
    assert "scaled from the N=1 counters" in roof["traffic_source"]


def test_fp8_mixed_mac_split():
    """bench.py's ceiling for the mixed fp8 kernel (mlp_fp8.hip, round 5): the MACs it runs on
    the bf16 MFMA (L0, L1, L4's encoding inputs, C0, both heads) and on the fp8 MFMA (L2, L3,
    L5-L7, L4's hidden inputs) add up to the network's, from the layer shapes."""
    import bench
    from oracle import nerf_oracle as O

    macs = {n: o * i for n, o, i in W.LAYER_SPECS}
    bf16 = sum(macs[n] for n in O.FP8_BF16_LAYERS) + 256 * W.POS_DIM + macs["density_head"] + macs["color_layers.1"]
    fp8 = sum(macs[f"layers.{i}"] for i in (2, 3, 5, 6, 7)) + 256 * 256
    assert bench.FP8_MIX_MACS == {"bf16": bf16, "fp8": fp8}
    assert bf16 + fp8 == W.MACS_PER_SAMPLE
    assert abs(bench.FP8_MIX_CEILING - 3983.8) < 0.1
