"""NeRFTrainer's training step on the MI355X.

``MI355XTrainer`` mirrors the reference's ``NeRFTrainer``
(``src/training/trainer.py:22-138``): the same configuration keys and defaults
(``:25-81``), ``train_step(batch) -> float`` with the batch dict of the synthetic
dataset (``src/data/loader.py:71-76``: image [H, W, 3], pose [4, 4], focal), the
loss history lists and a reference-format checkpoint (``:376-384``).  The step
itself is one call into the HIP library (``nerf_train_step``, include/nerf_mi355x.h):
rays, stratified coarse and uniform fine samples, both networks forward and
backward on the f32 MFMA, volume rendering with its backward, gradient clipping,
Adam and the lr schedule all run on the device.  Nothing is computed in PyTorch;
torch only provides device memory, the stream and the two random draws of a step
(``torch.randperm`` for the rays, ``torch.rand`` for the stratification), which can
also be injected for parity runs.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Mapping, Optional, Tuple

import numpy as np

from . import runtime as rt
from .weights import LAYER_SPECS, StateDict, save_checkpoint, synthetic_state_dict, validate_state_dict

# NeRFTrainer.__init__ defaults (trainer.py:50-75); main.py:25-61 overrides some of them
DEFAULTS = {
    "lr": 5e-4,
    "weight_decay": 0.0,
    "lr_decay": 0.1,
    "decay_steps": 250000,
    "n_coarse": 64,
    "n_fine": 128,
    "chunk_size": 1024,
    "near": 2.0,
    "far": 6.0,
    "gradient_clipping": None,
    "n_rays": 1024,
    "checkpoint_frequency": 50,
}


# Per-sample GEMM work of one net's training pass (train.hip gemm_macs_per_sample): the
# forward and weight-gradient GEMMs cover the 8 trunk layers, colour-0 and density
# (colour-1's 3 x 128 runs in the head kernels); backward-data skips the encodings' inputs.
GEMM_MACS_PER_SAMPLE = {"forward": 527_488, "backward_data": 7 * 256 * 256 + 129 * 256, "weight_grad": 527_488}
# Operand bytes the nine weight-gradient GEMMs read per sample, each GEMM's two row
# operands once (dW = dZ^T [X | PE]): head 128 + 283, layer 0 256 + 63, layer 4 256 + 319,
# six 256 x 256 layers; fp32.
WGRAD_OPERAND_BYTES_PER_SAMPLE = 4 * ((128 + 283) + (256 + 63) + (256 + 319) + 6 * 512)

# main.py:get_default_config (main.py:25-61), less the device key
MAIN_CONFIG = {
    "lr": 3e-4,
    "lr_decay": 0.1,
    "decay_steps": 250000,
    "n_rays": 2048,
    "n_coarse": 64,
    "n_fine": 128,
    "hidden_dim": 256,
    "position_encoding_levels": 10,
    "direction_encoding_levels": 4,
    "chunk_size": 1024,
    "near": 2.0,
    "far": 6.0,
    "gradient_clipping": 1.0,
    "weight_decay": 1e-6,
    "checkpoint_frequency": 25,
}


def _shapes():
    out = []
    for name, o, i in LAYER_SPECS:
        out.append((f"{name}.weight", (o, i)))
        out.append((f"{name}.bias", (o,)))
    return out


class MI355XTrainer:
    """NeRFTrainer on one MI355X: coarse + fine NeRFModel, one Adam over both, ExponentialLR."""

    def __init__(self, config: Dict, coarse: Optional[Mapping[str, np.ndarray]] = None,
                 fine: Optional[Mapping[str, np.ndarray]] = None, device_index: int = 0):
        import torch

        self.config = dict(DEFAULTS, **config)
        c = self.config
        if c.get("hidden_dim", 256) != 256 or c.get("position_encoding_levels", 10) != 10 or \
                c.get("direction_encoding_levels", 4) != 4:
            raise ValueError("the HIP kernels implement NeRFModel(pos_L=10, dir_L=4, hidden_dim=256)")
        # fresh models when no state dicts are given: nn.Linear's init distribution
        # (trainer.py:38-48 builds new NeRFModels)
        coarse = coarse if coarse is not None else synthetic_state_dict(0, conditioned=False)
        fine = fine if fine is not None else synthetic_state_dict(1, conditioned=False)
        validate_state_dict(coarse)
        validate_state_dict(fine)
        self.device = f"cuda:{device_index}"
        self.device_index = device_index
        self.n_coarse, self.n_fine = int(c["n_coarse"]), int(c["n_fine"])
        self.near, self.far = float(c["near"]), float(c["far"])
        self.chunk_size = int(c["chunk_size"])
        self.gradient_clipping = c["gradient_clipping"]
        self.checkpoint_frequency = c["checkpoint_frequency"]
        self.train_losses: list = []
        self.val_losses: list = []
        cfg = rt.TrainConfig()
        cfg.lr = float(c["lr"])
        cfg.beta1, cfg.beta2, cfg.eps = 0.9, 0.999, 1e-8
        cfg.weight_decay = float(c["weight_decay"])
        cfg.lr_gamma = float(c["lr_decay"]) ** (1 / c["decay_steps"])
        cfg.grad_clip = float(self.gradient_clipping) if self.gradient_clipping is not None else 0.0
        cfg.n_coarse, cfg.n_fine = self.n_coarse, self.n_fine
        cfg.near_, cfg.far_ = self.near, self.far
        self._cfg = cfg
        self.lib = rt.load_library()
        kc, pc = rt._param_list(coarse)
        kf, pf = rt._param_list(fine)
        h = ctypes.c_void_p()
        rt._check(self.lib.nerf_trainer_create(device_index, ctypes.byref(cfg), pc, pf, rt.NERF_N_PARAMS,
                                               ctypes.byref(h)))
        del kc, kf
        self._h = h
        # the forward's and backward-data chain's arithmetic ("fp32": the reference's;
        # "bf16x3": split bf16, faster, gradients as close to the float64 step as fp32's;
        # include/nerf_mi355x.h)
        self.precision = "fp32"
        try:
            self.set_precision(str(c.get("precision", "fp32")))
        except ValueError:
            self.close()
            raise
        self._loss = torch.zeros(3, dtype=torch.float32, device=self.device)
        self._grad_t = None
        self._render_dev = None      # inference context for render_image / validate

    def close(self) -> None:
        if getattr(self, "_render_dev", None) is not None:
            self._render_dev.close()
            self._render_dev = None
        if getattr(self, "_h", None) is not None and self._h.value:
            if getattr(self, "_grad_t", None) is not None:
                self.lib.nerf_trainer_set_grad_buffer(self._h, None)   # before the tensor goes
            self.lib.nerf_trainer_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ----------------------------------------------------------------- step --
    def draws(self, height: int, width: int, n_rays: int, generator=None):
        """The step's random draws as the reference makes them: torch.randperm over the
        pixels, first n_rays (trainer.py:111), and U[0,1) per coarse sample (rendering.py:47)."""
        import torch

        sel = torch.randperm(height * width, device=self.device, generator=generator)[:n_rays]
        t_rand = torch.rand(sel.numel(), self.n_coarse, device=self.device, generator=generator)
        return sel.to(torch.int32), t_rand

    def _inputs(self, batch: Mapping, select_inds, t_rand):
        """Device inputs of a step: image [H, W, 3], host pose [4, 4], focal, and the draws
        (made here as the reference makes them when not injected)."""
        import torch

        image = batch["image"]
        if not isinstance(image, torch.Tensor):
            image = torch.as_tensor(np.asarray(image, dtype=np.float32))
        image = image.to(self.device, torch.float32).contiguous()
        if image.dim() != 3 or image.shape[-1] != 3:
            raise ValueError(f"image must be [H, W, 3], got {tuple(image.shape)}")
        height, width = int(image.shape[0]), int(image.shape[1])
        pose = batch["pose"]
        pose = pose.detach().cpu().numpy() if hasattr(pose, "detach") else np.asarray(pose)
        pose = np.ascontiguousarray(pose.astype(np.float32).reshape(4, 4))
        focal = float(batch["focal"])
        n_rays = int(self.config["n_rays"])
        if select_inds is None or t_rand is None:
            s_draw, t_draw = self.draws(height, width, min(n_rays, height * width))
            select_inds = s_draw if select_inds is None else select_inds
            t_rand = t_draw if t_rand is None else t_rand
        sel = torch.as_tensor(select_inds).to(self.device, torch.int32).contiguous()
        tr = torch.as_tensor(t_rand).to(self.device, torch.float32).contiguous()
        if tuple(tr.shape) != (sel.numel(), self.n_coarse):
            raise ValueError(f"t_rand must be [{sel.numel()}, {self.n_coarse}], got {tuple(tr.shape)}")
        return image, pose, focal, sel, tr

    def train_step(self, batch: Mapping, select_inds=None, t_rand=None, update: bool = True,
                   sync: bool = True):
        """NeRFTrainer.train_step (trainer.py:83-138): returns the step's loss (a float, as
        loss.item(); with sync=False the device tensor [loss, mse_coarse, mse_fine])."""
        import torch

        image, pose, focal, sel, tr = self._inputs(batch, select_inds, t_rand)
        stream = torch.cuda.current_stream(self.device)
        rt._check(self.lib.nerf_train_step(self._h, image.data_ptr(), image.shape[0], image.shape[1], focal,
                                           rt._fptr(pose), sel.data_ptr(), sel.numel(), tr.data_ptr(),
                                           0 if update else rt.NERF_TRAIN_NO_UPDATE, self._loss.data_ptr(),
                                           int(stream.cuda_stream)))
        # keep the inputs alive until the queued step has consumed them
        self._keep = (image, sel, tr)
        if not sync:
            return self._loss
        return float(self._loss[0].item())

    def backward(self, batch: Mapping, select_inds, t_rand, n_rays_total: int):
        """This share's gradients of a step of n_rays_total rays (nerf_train_backward): the
        data-parallel half step; returns the device loss parts [loss, mse_c, mse_f]."""
        import torch

        image, pose, focal, sel, tr = self._inputs(batch, select_inds, t_rand)
        stream = torch.cuda.current_stream(self.device)
        rt._check(self.lib.nerf_train_backward(self._h, image.data_ptr(), image.shape[0], image.shape[1], focal,
                                               rt._fptr(pose), sel.data_ptr(), sel.numel(), int(n_rays_total),
                                               tr.data_ptr(), self._loss.data_ptr(), int(stream.cuda_stream)))
        self._keep = (image, sel, tr)
        return self._loss

    def grad_tensor(self):
        """The gradient store as a device tensor [2 * NERF_TRAIN_NET_FLOATS] (coarse then fine,
        state-dict order), so that torch.distributed can all-reduce it in place."""
        import torch

        if self._grad_t is None:
            t = torch.zeros(2 * rt.NERF_TRAIN_NET_FLOATS, dtype=torch.float32, device=self.device)
            rt._check(self.lib.nerf_trainer_set_grad_buffer(self._h, t.data_ptr()))
            self._grad_t = t
        return self._grad_t

    def update(self) -> None:
        """Clip + Adam + schedule on the current gradients (the last part of train_step)."""
        import torch

        rt._check(self.lib.nerf_trainer_update(self._h, int(torch.cuda.current_stream(self.device).cuda_stream)))

    # ---------------------------------------------------------------- state --
    def _read(self, what: int, net: int) -> StateDict:
        bufs = [np.zeros(shape, np.float32) for _, shape in _shapes()]
        ptrs = (rt._FP * rt.NERF_N_PARAMS)(*[rt._fptr(b) for b in bufs])
        rt._check(self.lib.nerf_trainer_read(self._h, what, net, ptrs, rt.NERF_N_PARAMS))
        return {name: b for (name, _), b in zip(_shapes(), bufs)}

    def state_dicts(self) -> Tuple[StateDict, StateDict]:
        """(coarse, fine) parameters as NeRFModel state dicts (host arrays)."""
        return self._read(rt.NERF_TR_PARAMS, 0), self._read(rt.NERF_TR_PARAMS, 1)

    def grads(self, net: int) -> StateDict:
        return self._read(rt.NERF_TR_GRADS, net)

    def exp_avg(self, net: int) -> StateDict:
        return self._read(rt.NERF_TR_EXP_AVG, net)

    def exp_avg_sq(self, net: int) -> StateDict:
        return self._read(rt.NERF_TR_EXP_AVG_SQ, net)

    def write_grads(self, net: int, grads: Mapping[str, np.ndarray]) -> None:
        keep, ptrs = rt._param_list(grads)
        rt._check(self.lib.nerf_trainer_write_grads(self._h, net, ptrs, rt.NERF_N_PARAMS))
        del keep

    def write(self, what: int, net: int, tensors: Mapping[str, np.ndarray]) -> None:
        """Overwrite one net's parameters / gradients / Adam moments (rt.NERF_TR_*)."""
        keep, ptrs = rt._param_list(tensors)
        rt._check(self.lib.nerf_trainer_write(self._h, what, net, ptrs, rt.NERF_N_PARAMS))
        del keep

    def set_schedule(self, steps: int, lr: float) -> None:
        """Adam's step count and the current learning rate."""
        rt._check(self.lib.nerf_trainer_set_schedule(self._h, int(steps), float(lr)))

    @property
    def lr(self) -> float:
        """optimizer.param_groups[0]['lr'] for the next step."""
        return float(self.lib.nerf_trainer_lr(self._h))

    @property
    def steps(self) -> int:
        return int(self.lib.nerf_trainer_steps(self._h))

    def set_precision(self, precision: str) -> None:
        """The arithmetic of the forward and the backward-data chain: "fp32" (the reference's)
        or "bf16x3" (split bf16 on the bf16 MFMA; nerf_trainer_set_precision in
        include/nerf_mi355x.h)."""
        if precision not in ("fp32", "bf16x3"):
            raise ValueError(f"precision {precision!r}: 'fp32' or 'bf16x3'")
        rt._check(self.lib.nerf_trainer_set_precision(self._h, rt.PRECISIONS[precision]))
        self.precision = precision

    def set_profiling(self, enable: bool) -> None:
        rt._check(self.lib.nerf_trainer_set_profiling(self._h, 1 if enable else 0))

    def stage_ms(self) -> Dict[str, float]:
        ms = (ctypes.c_float * rt.NERF_TRAIN_N_STAGES)()
        rt._check(self.lib.nerf_trainer_stage_ms(self._h, ms))
        return dict(zip(rt.TRAIN_STAGES, list(ms)))

    def gemm_flops(self) -> float:
        """Algorithmic fp32 FLOP of the last step's GEMMs."""
        return float(self.lib.nerf_trainer_gemm_flops(self._h))

    # ------------------------------------------------------------ epochs --
    def render_image(self, pose, img_shape, focal: float):
        """NeRFTrainer._render_image (trainer.py:353-371): every pixel's ray through the fine
        net at n_fine uniform samples (_render_rays' coarse result is discarded there) and
        volume_render, on the fp32 render path with the trainer's current fine weights (the
        same rays, z values and compositing as rendering.py); [H, W, 3] device tensor."""
        import torch

        h, w = int(img_shape[0]), int(img_shape[1])
        if self._render_dev is None:
            self._render_dev = rt.Device(self.device_index)
        self._render_dev.load_weights(rt.NERF_NET_FINE, self.state_dicts()[1])
        pose = pose.detach().cpu().numpy() if hasattr(pose, "detach") else np.asarray(pose)
        rgb = torch.empty(h, w, 3, dtype=torch.float32, device=self.device)
        depth = torch.empty(h, w, dtype=torch.float32, device=self.device)
        self._render_dev.render(np.asarray(pose, np.float32), w, h, 0, h, float(focal), self.near, self.far,
                                rt.linspace01(self.n_fine), 0, None, rt.NERF_FP32, rgb, depth,
                                stream=torch.cuda.current_stream(self.device))
        return rgb

    def validate(self, val_dataset) -> float:
        """NeRFTrainer.validate (trainer.py:140-170): mean MSE of the rendered image over the
        first five validation views."""
        import torch

        losses = []
        for i in range(min(5, len(val_dataset))):
            batch = val_dataset[i]
            image = torch.as_tensor(np.asarray(batch["image"].detach().cpu() if hasattr(batch["image"], "detach")
                                               else batch["image"], np.float32)).to(self.device)
            pred = self.render_image(batch["pose"], tuple(image.shape[:2]), float(batch["focal"]))
            losses.append(float(torch.mean((pred - image) ** 2).item()))
        return float(np.mean(losses))

    def train(self, train_dataset, val_dataset=None, n_epochs: int = 100, checkpoint_dir: str = "checkpoints"):
        """NeRFTrainer.train (trainer.py:172-244): resume from the latest
        checkpoint_epoch_<n>.pth in checkpoint_dir, then per epoch one train_step per image, the
        epoch's mean loss appended to train_losses, validate every 10th epoch, a checkpoint every
        checkpoint_frequency epochs."""
        import glob
        import os
        import re

        start = 0
        found = []
        for f in glob.glob(os.path.join(checkpoint_dir, "checkpoint_epoch_*.pth")):
            m = re.search(r"checkpoint_epoch_(\d+)\.pth$", f)
            if m:
                found.append((int(m.group(1)), f))
        if found:
            latest = max(found)[1]
            print(f"Found checkpoint: {latest}")
            self.load_checkpoint(latest)
            start = len(self.train_losses)
            print(f"Resuming training from epoch {start + 1}/{n_epochs}")
        else:
            print(f"No checkpoint found. Starting training from epoch 1/{n_epochs}")
        if start >= n_epochs:
            print(f"Training already completed! ({start}/{n_epochs} epochs)")
            return
        for epoch in range(start, n_epochs):
            losses = [self.train_step(train_dataset[i]) for i in range(len(train_dataset))]
            avg = float(np.mean(losses))
            self.train_losses.append(avg)
            if val_dataset is not None and (epoch + 1) % 10 == 0:
                val = self.validate(val_dataset)
                self.val_losses.append(val)
                print(f"Epoch {epoch + 1}: Train Loss = {avg:.4f}, Val Loss = {val:.4f}")
            else:
                print(f"Epoch {epoch + 1}: Train Loss = {avg:.4f}")
            if self.checkpoint_frequency and (epoch + 1) % int(self.checkpoint_frequency) == 0:
                self.save_checkpoint(os.path.join(checkpoint_dir, f"checkpoint_epoch_{epoch + 1}.pth"))
        print("Training completed!")

    def _torch_optimizer(self):
        """torch.optim.Adam + ExponentialLR over CPU stand-ins of the 44 parameters (coarse then
        fine, state-dict order: NeRFTrainer's `list(coarse.parameters()) + list(fine...)`,
        trainer.py:54-64) holding this trainer's state, for state_dict() in torch's format."""
        import torch

        c = self.config
        params = [torch.nn.Parameter(torch.from_numpy(v.copy()))
                  for sd in self.state_dicts() for v in sd.values()]
        opt = torch.optim.Adam(params, lr=float(c["lr"]), weight_decay=float(c["weight_decay"]))
        sched = torch.optim.lr_scheduler.ExponentialLR(opt, gamma=self._cfg.lr_gamma)
        steps = self.steps
        if steps > 0:
            moments = [(self.exp_avg(n), self.exp_avg_sq(n)) for n in (0, 1)]
            i = 0
            for net in (0, 1):
                for k in self.state_dicts()[net]:
                    opt.state[params[i]] = {"step": torch.tensor(float(steps)),
                                            "exp_avg": torch.from_numpy(moments[net][0][k].copy()),
                                            "exp_avg_sq": torch.from_numpy(moments[net][1][k].copy())}
                    i += 1
        opt.param_groups[0]["lr"] = self.lr
        sched.last_epoch = steps
        sched._step_count = steps + 1
        sched._last_lr = [self.lr]
        return opt, sched

    def save_checkpoint(self, path: str, full: bool = True) -> str:
        """NeRFTrainer.save_checkpoint (trainer.py:373-386): coarse_model, fine_model, optimizer
        and scheduler state dicts in torch's format, config and loss histories (a reference
        NeRFTrainer resumes from it with load_checkpoint); MI355XRenderer.setup reads the model
        entries.  full=False writes the model entries only."""
        coarse, fine = self.state_dicts()
        if not full:
            return save_checkpoint(path, coarse, fine)
        import os

        import torch

        opt, sched = self._torch_optimizer()
        ck = {"coarse_model": {k: torch.from_numpy(v) for k, v in coarse.items()},
              "fine_model": {k: torch.from_numpy(v) for k, v in fine.items()},
              "optimizer": opt.state_dict(), "scheduler": sched.state_dict(), "config": dict(self.config),
              "train_losses": list(self.train_losses), "val_losses": list(self.val_losses)}
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        torch.save(ck, path)
        return path

    def load_checkpoint(self, path: str) -> None:
        """NeRFTrainer.load_checkpoint (trainer.py:388-399): models, Adam's moments and step,
        the scheduler's learning rate and the loss histories, from a checkpoint written by the
        reference trainer or by save_checkpoint (loaded with weights_only=True, numpy scalars
        admitted: the reference's loss histories are np.float64, trainer.py:336-345)."""
        from .weights import torch_load_weights_only

        ck = torch_load_weights_only(path)
        sds = [{k: v.detach().cpu().numpy().astype(np.float32) for k, v in ck[name].items()}
               for name in ("coarse_model", "fine_model")]
        for net, sd in enumerate(sds):
            validate_state_dict(sd)
            self.write(rt.NERF_TR_PARAMS, net, sd)
        names = [list(sd.keys()) for sd in sds]
        opt = ck.get("optimizer")
        steps, lr = 0, float(self.config["lr"])
        if opt is not None:
            state = opt.get("state", {})
            lr = float(opt["param_groups"][0]["lr"])
            for which, key in ((rt.NERF_TR_EXP_AVG, "exp_avg"), (rt.NERF_TR_EXP_AVG_SQ, "exp_avg_sq")):
                for net in (0, 1):
                    t = {}
                    for j, k in enumerate(names[net]):
                        st = state.get(22 * net + j)
                        t[k] = (st[key].detach().cpu().numpy().astype(np.float32) if st is not None
                                else np.zeros_like(sds[net][k]))
                    self.write(which, net, t)
            steps = max([int(float(st["step"])) for st in state.values()] or [0])
        sched = ck.get("scheduler")
        if sched is not None and "_last_lr" in sched:
            lr = float(sched["_last_lr"][0])
        self.set_schedule(steps, lr)
        self.train_losses = [float(v) for v in ck.get("train_losses", [])]
        self.val_losses = [float(v) for v in ck.get("val_losses", [])]
