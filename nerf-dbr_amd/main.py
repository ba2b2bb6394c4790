"""CLI counterpart of the reference's ``main.py`` benchmark mode (``main.py:112-262``).

    python nerf-dbr_amd/main.py --benchmark_only --checkpoint checkpoints/final_model.pth

Same flags (``--data_dir --epochs --skip_training --checkpoint --benchmark_only``,
``main.py:202-217``) and the same default grid (200x150 / 400x300 / 800x600 x 32 / 64 /
128 spp, 2 views, ``main.py:134-141``).  Without ``--benchmark_only``/``--skip_training``
it trains first, as ``train_nerf`` does (``main.py:65-109``), with ``MI355XTrainer`` and
main.py's configuration on the Blender-format dataset in ``--data_dir``
(``nerf_amd.data.load_synthetic_data``, the contract of ``src/data/loader.py``).
``--lego-checkpoint`` writes the distilled Lego checkpoint (``nerf_amd.weights``) to
``--checkpoint`` first, ``--synthetic-checkpoint`` the deterministic conditioned one;
both only with ``--benchmark_only`` / ``--skip_training`` (they would replace the
trained model).
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="NeRF unified benchmark on MI355X")
    ap.add_argument("--data_dir", default="data/nerf_synthetic/lego")
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--skip_training", action="store_true")
    ap.add_argument("--checkpoint", default="checkpoints/final_model.pth")
    ap.add_argument("--benchmark_only", action="store_true")
    ap.add_argument("--synthetic-checkpoint", action="store_true",
                    help="write the deterministic synthetic checkpoint to --checkpoint first")
    ap.add_argument("--lego-checkpoint", action="store_true",
                    help="write the distilled Lego checkpoint to --checkpoint first")
    ap.add_argument("--resolutions", default="200x150,400x300,800x600")
    ap.add_argument("--spp", default="32,64,128")
    ap.add_argument("--views", type=int, default=2)
    ap.add_argument("--precisions", default="fp32,f16x3,bf16")
    ap.add_argument("--hierarchical", type=int, default=0, help="also run bf16 with N importance samples")
    ap.add_argument("--output_dir", default="outputs")
    args = ap.parse_args(argv)

    from nerf_amd import weights as W
    from nerf_amd.benchmark.benchmark_suite import UnifiedBenchmarkSuite

    train = not (args.skip_training or args.benchmark_only)
    if train and (args.synthetic_checkpoint or args.lego_checkpoint):
        ap.error("--synthetic-checkpoint / --lego-checkpoint replace the checkpoint: use them with "
                 "--benchmark_only or --skip_training")
    if args.synthetic_checkpoint and args.lego_checkpoint:
        ap.error("--synthetic-checkpoint and --lego-checkpoint are exclusive")
    if train:
        from nerf_amd.data import load_synthetic_data
        from nerf_amd.trainer import MAIN_CONFIG, MI355XTrainer

        datasets = load_synthetic_data(args.data_dir, "cpu")
        if "train" not in datasets:
            raise ValueError(f"Training dataset not found in {args.data_dir}")
        trainer = MI355XTrainer(dict(MAIN_CONFIG))
        trainer.train(datasets["train"], datasets.get("val"), args.epochs)
        trainer.save_checkpoint(args.checkpoint)
        print(f"\nTraining completed! Model saved to: {args.checkpoint}")
    if args.synthetic_checkpoint:
        W.write_synthetic_checkpoint(args.checkpoint)
    if args.lego_checkpoint:
        W.write_lego_checkpoint(args.checkpoint)
    if not os.path.exists(args.checkpoint):
        print(f"Error: Checkpoint not found at {args.checkpoint}")
        return 1
    res = [tuple(int(v) for v in r.split("x")) for r in args.resolutions.split(",")]
    spp = [int(s) for s in args.spp.split(",")]
    suite = UnifiedBenchmarkSuite(args.output_dir)
    suite.add_available_renderers(tuple(args.precisions.split(",")), args.hierarchical)
    if not suite.renderers:
        print("No renderers available for benchmarking!")
        return 1
    suite.run_benchmark(args.checkpoint, res, spp, args.views)
    df = suite.generate_report()
    if not df.empty:
        print(df.to_string(index=False))
    return 0


if __name__ == "__main__":
    sys.exit(main())
