"""Which torch ops launch the small element-wise / copy kernels of a training step (the "glue" between the HIP
kernels): one bench workload, warm-up steps, then one step under torch.profiler; prints the aten ops that own
device kernels, with call counts, device time and input shapes, and the python frames that issued the most.

usage: python scripts/prof_glue.py --model sv [bench.py options]"""
import collections
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402
from torch.profiler import profile, ProfilerActivity  # noqa: E402

import bench  # noqa: E402
from viforssms_amd import _lib  # noqa: E402
from viforssms_amd.launch import init_distributed  # noqa: E402


def main():
    args = bench.parse_args(sys.argv[1:])
    ctx = init_distributed()
    dev = torch.device("cuda", torch.cuda.current_device())
    model, _ = bench.build_model(args, ctx, dev, _lib.TRAIN_PRECISIONS[args.precision])
    for i in range(3):
        model.elbo_step(model.batch_for(model.select_windows()), i)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        model.elbo_step(model.batch_for(model.select_windows()), 3)
        torch.cuda.synchronize()
    skip = ("vissm", "hip", "Memcpy", "Memset")
    rows = []
    for e in prof.key_averages(group_by_input_shape=True):
        dt = getattr(e, "device_time_total", 0) or getattr(e, "cuda_time_total", 0)
        if e.key.startswith("aten::") and dt > 0:
            rows.append((e.count, dt, e.key, str(e.input_shapes)[:120]))
    rows.sort(key=lambda r: -r[0])
    print(f"{'calls':>5} {'dev us':>8}  op  shapes")
    for c, t, k, s in rows[:40]:
        print(f"{c:5d} {t:8.0f}  {k}  {s}")
    frames = collections.Counter()
    for e in prof.events():
        if e.name in ("aten::add_", "aten::add", "aten::copy_", "aten::fill_", "aten::zero_", "aten::mul", "aten::cat",
                      "aten::stack", "aten::sum", "aten::mul_", "aten::neg", "aten::sub", "aten::div", "aten::zeros"):
            st = [f for f in (e.stack or []) if "viforssms_amd" in f or "bench" in f]
            frames[(e.name, st[0] if st else "(autograd engine)")] += 1
    print("\nissuing frames (op, first repo frame): calls")
    for (op, fr), n in frames.most_common(30):
        print(f"{n:5d}  {op:14s} {fr}")
    _ = skip


if __name__ == "__main__":
    main()
