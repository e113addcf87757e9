"""hyperparameters.txt format and the main.py command line (main.py:6-57, 59-130 of the reference).

The file is read positionally: values sit at 0-based line indices 1, 3, ..., 27 in the order
T, impute, x0, theta, obs_std, p, kernel_len, batch_dims, network_dims, no_flows, priors,
feat_window, learn_rate, grad_clip.  Command-line overrides win over the file.  Extra flags of
this build (not in the reference): -p/-samples, --gpus, --steps, --seed, --precision, --no-pretrain.
"""
from __future__ import annotations

import argparse
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

DEFAULT_FILE = """#### T ####
5000
#### impute ####
1
#### x0 ####
10.0
#### Theta ####
5.0, 0.5, 3.0
#### Observation Standard Deviation ####
1.
#### p ####
50
#### kernel_len ####
50
#### batch_dims ####
50
#### network_dims ####
50, 50, 50
#### no_flows ####
3
####  priors ####
(0., 10.0)(0., 10.0)(0., 10.0)
#### feat_window ####
10
#### learn_rate ####
1e-3
#### grad_clip ####
2.5e8
"""


@dataclass
class HyperParams:
    T: int
    impute: int
    x0: float
    theta: List[float]
    obs_std: float
    p: int
    kernel_len: int
    batch_dims: int
    network_dims: List[int]
    no_flows: int
    priors: List[Tuple[float, float]]
    feat_window: int
    learn_rate: float
    grad_clip: float


def parse_priors(line: str) -> List[Tuple[float, float]]:
    parts = line.rstrip().replace(")", "").split("(")[1:]
    return [(float(t.split(",")[0]), float(t.split(",")[1])) for t in parts]


def parseparams(file) -> list:
    """Positional parse (reference main.py:26-57); returns the 14 values as a list."""
    with open(file, "r") as f:
        lines = f.readlines()
    vals = [
        int(lines[1].rstrip()),
        int(lines[3].rstrip()),
        float(lines[5].rstrip()),
        [float(t) for t in lines[7].rstrip().split(",")],
        float(lines[9].rstrip()),
        int(lines[11].rstrip()),
        int(lines[13].rstrip()),
        int(lines[15].rstrip()),
        [int(d) for d in lines[17].rstrip().split(",")],
        int(lines[19].rstrip()),
        parse_priors(lines[21]),
        int(lines[23].rstrip()),
        float(lines[25].rstrip()),
        float(lines[27].rstrip()),
    ]
    return vals


def to_hparams(vals: list) -> HyperParams:
    return HyperParams(*vals)


def handle_opts(argv=None):
    parser = argparse.ArgumentParser(
        formatter_class=argparse.RawDescriptionHelpFormatter,
        description="Neural moving-average variational inference for SDEs on MI355X (AR(1) driver).",
        usage="%(prog)s hyperparameters.txt [OPTIONS] \n Any options passed will be prioritised over the setting "
              "in the hyperparameters text file. \n To repair your hyperparameters file use -repair and copy and "
              "paste the output into hyperparameters.txt")
    parser.add_argument("file", action="store", nargs="?", default=None, help="File containing all hyperparameters")
    parser.add_argument("-T", "-time", action="store", dest="T", default=None, help="Time")
    parser.add_argument("-i", "-impute", action="store", dest="impute", default=None, help="Impute")
    parser.add_argument("-t", "-theta", action="append", dest="theta", default=None, help="Theta values listed")
    parser.add_argument("-x", "-xzero", action="store", dest="x0", default=None, help="Value for x at time 0")
    parser.add_argument("-o", "-obs_std", action="store", dest="obs_std", default=None,
                        help="Observation standard deviation")
    parser.add_argument("-k", "-kernel_len", action="store", dest="kernel_len", default=None, help="Length of Kernel")
    parser.add_argument("-b", "-batch_dims", action="store", dest="batch_dims", default=None,
                        help="Batch Dimensions (window length M)")
    parser.add_argument("-f", "-feat_window", action="store", dest="feat_window", default=None, help="Feature Window")
    parser.add_argument("-repair", action="store_true", dest="repair", default=False,
                        help="Output default hyperparameters to repair file")
    # additions of this build
    parser.add_argument("-p", "-samples", action="store", dest="p", default=None,
                        help="Samples (windows) per step; overrides the file's p")
    parser.add_argument("--gpus", type=int, default=None,
                        help="Ranks (one per GPU): without torchrun, N > 1 launches N ranks itself; under torchrun "
                             "the launched world must equal N.  Default: the launcher's world (1 without one)")
    parser.add_argument("--steps", type=int, default=None, help="Stop after this many runs (default: endless)")
    parser.add_argument("--seed", type=int, default=1, help="Philox seed of the base noise")
    parser.add_argument("--precision", choices=["fp32", "bf16", "bf16x2", "bf16x3", "bf16x3f", "bf16x2f"],
                        default="fp32",
                        help="flow products: fp32 exact, bf16, bf16x2 (split weights, bf16 activations, forward and "
                             "backward), bf16x3 (split operands); bf16x3f / bf16x2f: "
                             "bf16x3 / split-weight forward products with bf16 backward products")
    parser.add_argument("--no-pretrain", action="store_true", help="Skip the 501 pre-training runs")
    parser.add_argument("--log-every", type=int, default=1)
    parser.add_argument("--graph", action="store_true",
                        help="Run the ELBO steps as a captured HIP graph (launch-bound small configs)")
    return parser.parse_args(argv)


def apply_overrides(hp: HyperParams, args) -> HyperParams:
    """main.py:112-128 (theta values are parsed as floats here; the reference keeps strings, a bug)."""
    if args.T is not None:
        hp.T = int(args.T)
    if args.impute is not None:
        hp.impute = int(args.impute)
    if args.theta is not None:
        vals = []
        for t in args.theta:
            vals += [float(v) for v in str(t).split(",") if v.strip()]
        hp.theta = vals
    if args.x0 is not None:
        hp.x0 = float(args.x0)
    if args.obs_std is not None:
        hp.obs_std = float(args.obs_std)
    if args.kernel_len is not None:
        hp.kernel_len = int(args.kernel_len)
    if args.batch_dims is not None:
        hp.batch_dims = int(args.batch_dims)
    if args.feat_window is not None:
        hp.feat_window = int(args.feat_window)
    if getattr(args, "p", None) is not None:
        hp.p = int(args.p)
    return hp
