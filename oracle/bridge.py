"""Checker-side glue: maps the product's named variables (viforssms_amd ParamStore) onto the
oracle's parameter dict and back, and builds the oracle ModelSpec from a product ModelDef.
TEST INFRASTRUCTURE ONLY (see nma_oracle.py header)."""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch

from . import nma_oracle as O


def spec_from_mdef(mdef, p: int) -> O.ModelSpec:
    return O.ModelSpec(family=mdef.family, p=p, M=mdef.M, k=mdef.k, n_flows=mdef.n_flows,
                       H=mdef.network_dims[0], n_layers=len(mdef.network_dims), C_time=mdef.C_time,
                       P_theta=mdef.P_theta, target=mdef.scale_num, priors=list(mdef.priors), dt=mdef.dt,
                       obs_std=mdef.obs_std, theta_act=mdef.theta_act, base_loc=mdef.theta_base[0],
                       base_scale=mdef.theta_base[1], n_maf=mdef.n_maf)


def _name_map(spec: O.ModelSpec) -> Dict[str, tuple]:
    """product name -> ("flow", i, oracle key) | ("maf", i, j, "w"|"b")."""
    m = {}
    for i in range(spec.n_flows):
        pre = f"flow{i}/"
        for j in range(4):
            m[pre + f"feat{j}/kernel"] = ("flow", i, f"feat_w{j}")
            m[pre + f"feat{j}/bias"] = ("flow", i, f"feat_b{j}")
        m[pre + "conv/kernel"] = ("flow", i, "conv_w")
        m[pre + "conv/bias"] = ("flow", i, "conv_b")
        for j in range(3):
            m[pre + f"theta{j}/kernel"] = ("flow", i, f"th_w{j}")
            m[pre + f"theta{j}/bias"] = ("flow", i, f"th_b{j}")
        for l in range(spec.n_layers - 2):
            m[pre + f"hidden{l}/kernel"] = ("flow", i, f"hid_w{l}")
            m[pre + f"hidden{l}/bias"] = ("flow", i, f"hid_b{l}")
            m[pre + f"bn{l}/gamma"] = ("flow", i, f"bn_g{l}")
            m[pre + f"bn{l}/beta"] = ("flow", i, f"bn_b{l}")
        m[pre + "head/kernel"] = ("flow", i, "head_w")
        m[pre + "head/bias"] = ("flow", i, "head_b")
    for i in range(spec.n_maf):
        for j in range(4):
            m[f"theta/maf{i}/dense{j}/kernel"] = ("maf", i, j, 0)
            m[f"theta/maf{i}/dense{j}/bias"] = ("maf", i, j, 1)
    return m


def oracle_params(values: Dict[str, np.ndarray], spec: O.ModelSpec, masks: List[np.ndarray],
                  dtype=O.DT) -> dict:
    """Builds the oracle params dict from product variable values (numpy, by product name)."""
    nm = _name_map(spec)
    flows = [dict() for _ in range(spec.n_flows)]
    mafs = [[[None, None, torch.tensor(masks[j], dtype=dtype)] for j in range(len(masks))] for _ in range(spec.n_maf)]
    for name, v in values.items():
        key = nm[name]
        t = torch.tensor(np.asarray(v, dtype=np.float64), dtype=dtype)
        if key[0] == "flow":
            flows[key[1]][key[2]] = t
        else:
            mafs[key[1]][key[2]][key[3]] = t
    return {"flows": flows, "mafs": [[tuple(l) for l in layers] for layers in mafs]}


def oracle_grads_by_name(params: dict, grads: List[torch.Tensor], spec: O.ModelSpec) -> Dict[str, np.ndarray]:
    """Maps train_step()'s gradient list (param_leaves order) back to product names."""
    leaves = O.param_leaves(params)
    ids = {id(t): g for t, g in zip(leaves, grads)}
    out = {}
    for name, key in _name_map(spec).items():
        if key[0] == "flow":
            t = params["flows"][key[1]].get(key[2])
        else:
            t = params["mafs"][key[1]][key[2]][key[3]]
        if t is not None and id(t) in ids:
            out[name] = ids[id(t)].detach().numpy()
    return out
