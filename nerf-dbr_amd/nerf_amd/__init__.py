"""nerf_amd: the NeRF render path of dgsmith7/nerf-dbr on MI355X (gfx950) HIP kernels.

weights      -- NeRFModel state-dict schema, checkpoints, the synthetic checkpoint
runtime      -- ctypes binding of libnerf_mi355x.so (include/nerf_mi355x.h)
distributed  -- row-band sharding + RCCL all-gather across one node's GPUs
benchmark    -- plugin interface, MI355XRenderer, benchmark suite
"""
__version__ = "0.1.0"
