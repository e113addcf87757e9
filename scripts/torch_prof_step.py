"""Op-level breakdown of the benchmarked training step (torch.profiler on the GPU): which torch ops
around the HIP kernels cost device time, grouped by op and input shape.
usage: python scripts/torch_prof_step.py [--model ar|lv|sv|fhn] [--precision bf16] [--rows 40]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--model", default="ar")
    ap.add_argument("--rows", type=int, default=45)
    a = ap.parse_args()
    args = bench.parse_args(["--precision", a.precision, "--model", a.model])
    from viforssms_amd import _lib
    from viforssms_amd.launch import init_distributed
    ctx = init_distributed()
    dev = torch.device("cuda", 0)
    model, _ = bench.build_model(args, ctx, dev, _lib.TRAIN_PRECISIONS[a.precision])

    def step(i):
        model.elbo_step(model.batch_for(model.select_windows()), i)

    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        for i in range(2):
            step(3 + i)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by="device_time_total", row_limit=a.rows, max_name_column_width=40,
                   max_shapes_column_width=70))


if __name__ == "__main__":
    main()
