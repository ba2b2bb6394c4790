"""Image-row-band sharding across the GPUs of one node, one process per GPU.

Rays are independent and cost the same (fixed samples per ray), so the frame
is cut into contiguous row bands, rank r rendering rows
``[floor(r*H/P), floor((r+1)*H/P))``.  Each rank renders its band
straight into a packed ``[rows, W, 4]`` fp32 tile (RGB + depth,
``nerf_render_band``), and the only exchange is one gather of those tiles to
the root over RCCL/xGMI (backend "nccl" on ROCm): 960 KB per rank at 800x600 on
8 GPUs, each rank's tile on its own direct xGMI link to the root.  An
all-gather (every rank receives the frame) is kept as an option.  The reference
has no distributed path at all; this replaces nothing and adds the multi-GPU
mode the benchmark reports.
"""
from __future__ import annotations

from typing import Callable, List, Tuple


def band(rank: int, world: int, height: int) -> Tuple[int, int]:
    return (rank * height) // world, ((rank + 1) * height) // world


def bands(world: int, height: int) -> List[Tuple[int, int]]:
    return [band(r, world, height) for r in range(world)]


def max_band_rows(world: int, height: int) -> int:
    return max(r1 - r0 for r0, r1 in bands(world, height))


_GATHER_BUFS = {}


def _gather_buffers(world: int, rows: int, width: int, device):
    """Send/receive buffers of gather_bands, allocated once per shape and device
    (a frame loop then launches no allocations)."""
    import torch

    key = (world, rows, width, str(device))
    if key not in _GATHER_BUFS:
        _GATHER_BUFS[key] = (torch.zeros(rows, width, 4, dtype=torch.float32, device=device),
                             torch.empty(world * rows, width, 4, dtype=torch.float32, device=device))
    return _GATHER_BUFS[key]


def band_tile(world: int, height: int, width: int, device):
    """The cached packed send tile of this shape ([max band rows, W, 4]); a rank
    renders its band into its first rows (nerf_render_band)."""
    rows = max_band_rows(world, height)
    key = ("tile", world, rows, width, str(device))
    if key not in _GATHER_BUFS:
        import torch

        _GATHER_BUFS[key] = torch.zeros(rows, width, 4, dtype=torch.float32, device=device)
    return _GATHER_BUFS[key]


def gather_tiles_to_root(tile, width: int, height: int, root: int = 0, group=None, copy: bool = False):
    """Gather every rank's packed band tile ([max rows, W, 4]) to `root`: one
    ``dist.gather`` (RCCL: the root receives from each rank on its own xGMI link).
    Returns the frame as a packed [H, W, 4] tensor on the root (its views
    [..., :3] and [..., 3] are the RGB and depth images), None elsewhere.

    With ``copy=False`` (the frame loop's form: no allocation per frame) the result
    ALIASES a receive buffer cached per shape whenever H divides evenly over the
    ranks: it is valid until the next gather of the same shape, which overwrites it.
    ``copy=True`` returns a tensor of its own in every case."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    rows = tile.shape[0]
    key = ("full", world, rows, width, str(tile.device))
    if key not in _GATHER_BUFS:
        _GATHER_BUFS[key] = torch.empty(world, rows, width, 4, dtype=torch.float32, device=tile.device)
    full = _GATHER_BUFS[key]
    if tile.is_cuda and dist.get_backend(group) == "gloo":
        # rehearsal of the multi-rank path on one device (gloo gathers host tensors)
        host = [torch.empty(rows, width, 4) for _ in range(world)] if rank == root else None
        dist.gather(tile.cpu(), host, dst=root, group=group)
        if rank == root:
            for r in range(world):
                full[r].copy_(host[r])
    else:
        dist.gather(tile, list(full.unbind(0)) if rank == root else None, dst=root, group=group)
    if rank != root:
        return None
    if height % world == 0:
        frame = full.reshape(world * rows, width, 4)
        return frame.clone() if copy else frame
    return torch.cat([full[r, : b1 - b0] for r, (b0, b1) in enumerate(bands(world, height))], 0)


def gather_bands(rgb_band, depth_band, width: int, height: int, group=None):
    """All-gather every rank's band into the full (rgb [H,W,3], depth [H,W]) on every rank
    (the option beside gather_tiles_to_root; it packs the separate rgb/depth bands first).

    Bands are padded to the largest band so one ``all_gather_into_tensor`` moves them
    (with H divisible by the world size, as 600 rows over 1/2/4/8 GPUs, there is no
    padding and the gathered buffer is the frame as it stands).
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    r0, r1 = band(rank, world, height)
    rows = max_band_rows(world, height)
    packed, full = _gather_buffers(world, rows, width, rgb_band.device)
    packed[: r1 - r0, :, :3] = rgb_band
    packed[: r1 - r0, :, 3] = depth_band
    if packed.is_cuda and dist.get_backend(group) == "gloo":
        # rehearsal of the multi-rank path on one device (gloo has no device
        # all-gather): stage through host memory
        host = torch.empty(world * rows, width, 4, dtype=torch.float32)
        dist.all_gather_into_tensor(host, packed.cpu(), group=group)
        full.copy_(host)
    else:
        dist.all_gather_into_tensor(full, packed, group=group)
    if height % world == 0:
        img = full
    else:
        full4 = full.reshape(world, rows, width, 4)
        img = torch.cat([full4[r, : b1 - b0] for r, (b0, b1) in enumerate(bands(world, height))], 0)
    return img[..., :3].contiguous(), img[..., 3].contiguous()


def init_from_env():
    """(rank, world, local, device index) from torchrun's environment; joins the
    process group when world > 1, or at world 1 when NERF_DIST_FORCE_GROUP=1 (the
    RCCL check on a one-GPU box: tests/test_gpu_parity.py).  Backend RCCL ("nccl")
    unless NERF_DIST_BACKEND says otherwise (gloo: the one-device rehearsal, ranks
    sharing device local % device_count)."""
    import os

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    if world > 1 or os.environ.get("NERF_DIST_FORCE_GROUP") == "1":
        backend = os.environ.get("NERF_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    return rank, world, local, dev


def reduce_max(x: float) -> float:
    """Max over ranks of a host float (the bench's max-over-ranks time)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return x
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def render_frame_to_root(renderer, camera_pose, resolution: Tuple[int, int], samples_per_ray: int,
                         root: int = 0, group=None):
    """This rank renders its band into the packed tile (renderer.render_band) and the
    tiles are gathered to `root`: (rgb [H,W,3], depth [H,W]) on the root, None elsewhere.
    The two are views of a frame tensor of their own (a later frame does not
    overwrite them)."""
    import torch.distributed as dist

    width, height = resolution
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    r0, r1 = band(rank, world, height)
    tile = band_tile(world, height, width, renderer.torch_device())
    renderer.render_band(camera_pose, resolution, samples_per_ray, r0, r1, tile)
    full = gather_tiles_to_root(tile, width, height, root, group, copy=True)
    return None if full is None else (full[..., :3], full[..., 3])


def render_sharded(render_rows: Callable, camera_pose, resolution: Tuple[int, int], samples_per_ray: int,
                   group=None, gather: bool = True):
    """Render this rank's band with ``render_rows(pose, res, spp, row0, row1)`` and all-gather."""
    import torch.distributed as dist

    width, height = resolution
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    r0, r1 = band(rank, world, height)
    rgb, depth = render_rows(camera_pose, resolution, samples_per_ray, r0, r1)
    if not gather:
        return rgb, depth
    return gather_bands(rgb, depth, width, height, group)


def train_step_sharded(trainer, batch, select, t_rand, group=None):
    """One NeRFTrainer.train_step (trainer.py:83-138) over the ranks of ``group``, data
    parallel.  Every rank holds the same step draw (select [n], t_rand [n, n_coarse]) and
    takes the contiguous share ``band(rank, world, n)`` of its rays; ``trainer.backward``
    returns that share's gradients with the loss normalised over all n rays, so one
    all-reduce (SUM) of the gradient store is the whole step's gradient (RCCL on ROCm,
    2 x 530,052 floats = 4.2 MB).  Clip, Adam and the schedule then run on every rank on
    identical gradients, so the replicas stay identical.  Returns the device tensor
    [loss, mse_coarse, mse_fine] of the whole step (all-reduced)."""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    n = int(select.shape[0])
    if n < world:
        raise ValueError(f"{n} rays cannot be shared by {world} ranks")
    a, b = band(rank, world, n)
    grads = trainer.grad_tensor()
    loss = trainer.backward(batch, select[a:b], t_rand[a:b], n_rays_total=n)
    if dist.is_initialized():
        dist.all_reduce(grads, group=group)
        dist.all_reduce(loss, group=group)
    trainer.update()
    return loss
