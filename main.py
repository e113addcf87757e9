"""Drop-in for the reference's ``python main.py hyperparameters.txt [OPTIONS]`` (AR(1) driver).

Same file format, flags and order of numpy-RNG draws as the reference main.py: the seed is set
when the data generator and the model modules are imported (AR_dat_gen.py:3, AR.py:18), then
data_gen writes dat/AR_*.txt, AR.main draws the q(theta) permutations and the training loop
draws the windows.  The ELBO step itself runs on the GPU (libvissm HIP kernels).
Multi-GPU: ``torchrun --nproc-per-node N main.py hyperparameters.txt -p P`` (or ``python main.py
hyperparameters.txt -p P --gpus N``, which launches the N ranks itself) shards the p samples.
"""
import os
import sys

import numpy as np

np.random.seed(1)  # import of AR_dat_gen (AR_dat_gen.py:3)
np.random.seed(1)  # import of AR (AR.py:18)

from viforssms_amd.config import DEFAULT_FILE, apply_overrides, handle_opts, parseparams, to_hparams  # noqa: E402


def run(argv=None):
    args = handle_opts(argv)
    if args.repair:
        print(DEFAULT_FILE)
        sys.exit("Copy the above into a .txt file")
    if not args.file:
        sys.exit("Please specify a valid hyperparameter file")
    try:
        hp = to_hparams(parseparams(args.file))
    except Exception:
        sys.exit("Please specify a valid hyperparameter file")
    hp = apply_overrides(hp, args)

    from viforssms_amd.launch import barrier, ensure_world, init_distributed
    if args.gpus is not None:
        rc = ensure_world(args.gpus, os.path.abspath(__file__), sys.argv[1:] if argv is None else list(argv))
        if rc is not None:
            sys.exit(rc)

    from viforssms_amd import ar
    from viforssms_amd._lib import TRAIN_PRECISIONS
    from viforssms_amd.data import data_gen

    ctx = init_distributed()
    data_gen(hp.T, hp.impute, hp.x0, np.array(hp.theta), hp.obs_std, write=(ctx.rank == 0))
    barrier(ctx)
    prec = TRAIN_PRECISIONS[args.precision]
    return ar.main(hp.p, hp.kernel_len, hp.T, hp.batch_dims, hp.network_dims, hp.no_flows, hp.priors,
                   hp.feat_window, hp.x0, hp.obs_std, learn_rate=hp.learn_rate, grad_clip=hp.grad_clip,
                   max_runs=args.steps, precision=prec, dist=ctx, seed=args.seed, pre_train=not args.no_pretrain,
                   log_every=args.log_every, graph=args.graph)


if __name__ == "__main__":
    run()
