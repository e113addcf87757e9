"""Probe for tests/test_launch.py: `python tests/_launch_probe.py --gpus N OUTDIR` goes through the same
launcher as bench.py / main.py (viforssms_amd.launch.ensure_world); every rank writes OUTDIR/rank<r>.txt with
"rank world" after a gloo all-reduce over the world (CPU host: init_distributed picks gloo)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("out")
    args = ap.parse_args()
    from viforssms_amd.launch import ensure_world, init_distributed
    rc = ensure_world(args.gpus, os.path.abspath(__file__), sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    import torch
    ctx = init_distributed()
    t = torch.ones(1)
    ctx.all_reduce_(t)
    with open(os.path.join(args.out, f"rank{ctx.rank}.txt"), "w") as f:
        f.write(f"{ctx.rank} {ctx.world} {int(t.item())}\n")


if __name__ == "__main__":
    main()
