"""Model / optimizer state-dict helpers for sharded checkpoints.

Same contract as `torch.distributed.checkpoint.state_dict` (SURVEY §5.4 "Helpers",
T/distributed/checkpoint/state_dict.py:93-135): the model state dict uses clean FQNs (no
`module.` prefix from a DDP wrapper), and the optimizer state dict is keyed by parameter
FQN instead of the process-local integer ids of `Optimizer.state_dict()` - ids are not
stable across model constructions, FQNs are, so a sharded `.metadata` written by one job
loads into another.  `get_state_dict` materialises lazily-created optimizer state first, so
the returned dict is a complete load target for `dcp.load` (which fills tensors in place).
Under ZeRO-1 the fused optimizers' state values are `FlatShardedTensor`s over this rank's
compact shards (checkpoint/sharded.py): `dcp.save` writes them as chunks and `dcp.load` reads
only the intersecting bytes, so a sharded checkpoint never all-gathers the optimizer state.

    model_sd, optim_sd = get_state_dict(model, opt)
    dcp.save({"model": model_sd, "optim": optim_sd}, path)
    ...
    model_sd, optim_sd = get_state_dict(model, opt)          # templates
    sd = {"model": model_sd, "optim": optim_sd}; dcp.load(sd, path)
    set_state_dict(model, opt, model_state_dict=sd["model"], optim_state_dict=sd["optim"])
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable

import torch
import torch.nn as nn


@dataclass
class StateDictOptions:
    full_state_dict: bool = False      # replicated DDP models are already full on every rank
    cpu_offload: bool = False          # return host copies (e.g. to hand to torch.save)
    strict: bool = True
    broadcast_from_rank0: bool = False  # set_*: only rank 0 holds real values; broadcast them


def _unwrap(model: nn.Module) -> nn.Module:
    return model.module if hasattr(model, "module") and isinstance(model.module, nn.Module) else model


def _fqns(model: nn.Module) -> dict:
    return {p: n for n, p in _unwrap(model).named_parameters()}


def _optims(optimizers) -> list:
    if optimizers is None:
        return []
    if isinstance(optimizers, torch.optim.Optimizer):
        return [optimizers]
    return list(optimizers)


def _maybe_cpu(sd, opts: StateDictOptions):
    if not opts.cpu_offload:
        return sd
    if torch.is_tensor(sd):
        return sd.detach().cpu()
    if isinstance(sd, dict):
        return {k: _maybe_cpu(v, opts) for k, v in sd.items()}
    if isinstance(sd, list):
        return [_maybe_cpu(v, opts) for v in sd]
    return sd


def get_model_state_dict(model: nn.Module, *, options: StateDictOptions | None = None) -> dict:
    opts = options or StateDictOptions()
    return _maybe_cpu(dict(_unwrap(model).state_dict()), opts)


def _init_optim_state(opt: torch.optim.Optimizer) -> None:
    if hasattr(opt, "init_state"):
        opt.init_state()
        return
    # stock torch optimizers: a step with zero gradients and lr 0 creates the state lazily
    saved = []
    for g in opt.param_groups:
        saved.append(g["lr"])
        g["lr"] = 0.0
        for p in g["params"]:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
    opt.step()
    opt.zero_grad(set_to_none=True)
    for g, lr in zip(opt.param_groups, saved):
        g["lr"] = lr


def get_optimizer_state_dict(model: nn.Module, optimizers, *, options: StateDictOptions | None = None) -> dict:
    opts = options or StateDictOptions()
    names = _fqns(model)
    state, groups = {}, []
    for opt in _optims(optimizers):
        if any(p not in opt.state for g in opt.param_groups for p in g["params"]):
            _init_optim_state(opt)
        if hasattr(opt, "_materialize_steps"):
            opt._materialize_steps()  # fused optimizers keep step counts as host ints
        for g in opt.param_groups:
            pg = {k: v for k, v in g.items() if k != "params"}
            pg["params"] = [names[p] for p in g["params"]]
            groups.append(pg)
            for p in g["params"]:
                st = opt.state.get(p)
                if st:
                    d = dict(st)
                    if hasattr(opt, "checkpoint_value"):
                        # ZeRO-1: FlatShardedTensor shards, written as DCP chunks (no all-gather)
                        d = {k: opt.checkpoint_value(p, k, v) for k, v in d.items()}
                    state[names[p]] = d
    return _maybe_cpu({"state": state, "param_groups": groups}, opts)


def get_state_dict(model: nn.Module, optimizers=None, *, options: StateDictOptions | None = None):
    return (get_model_state_dict(model, options=options),
            get_optimizer_state_dict(model, optimizers, options=options) if optimizers is not None else {})


def _broadcast_tree(sd, src: int = 0):
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    if torch.is_tensor(sd):
        dist.broadcast(sd, src)
    elif isinstance(sd, dict):
        for k in sorted(sd, key=str):
            _broadcast_tree(sd[k], src)


def set_model_state_dict(model: nn.Module, model_state_dict: dict, *, options: StateDictOptions | None = None):
    opts = options or StateDictOptions()
    m = _unwrap(model)
    if opts.broadcast_from_rank0:
        own = m.state_dict()
        with torch.no_grad():
            for k, v in model_state_dict.items():
                if k in own and torch.is_tensor(v):
                    own[k].copy_(v)
        _broadcast_tree(own)
        return None
    return m.load_state_dict(model_state_dict, strict=opts.strict)


def set_optimizer_state_dict(model: nn.Module, optimizers, optim_state_dict: dict, *,
                             options: StateDictOptions | None = None) -> None:
    """Load an FQN-keyed optimizer state dict: each current param group takes its
    hyper-parameters from the saved group at the same position, and every parameter takes the
    saved state stored under its FQN (so parameter order inside a group may differ)."""
    opts = options or StateDictOptions()
    names = _fqns(model)
    gi = 0
    for opt in _optims(optimizers):
        groups, state, nid = [], {}, 0
        for g in opt.param_groups:
            saved = optim_state_dict["param_groups"][gi]
            gi += 1
            cur = [names[p] for p in g["params"]]
            if sorted(cur) != sorted(saved["params"]):
                raise ValueError(f"optimizer param group {gi - 1} holds different parameters than the checkpoint")
            pg = {k: v for k, v in saved.items() if k != "params"}
            pg["params"] = list(range(nid, nid + len(cur)))
            for i, name in zip(pg["params"], cur):
                st = optim_state_dict["state"].get(name)
                if st is not None:
                    state[i] = st
            nid += len(cur)
            groups.append(pg)
        if opts.broadcast_from_rank0:
            _broadcast_tree(state)
        opt.load_state_dict({"state": state, "param_groups": groups})


def set_state_dict(model: nn.Module, optimizers=None, *, model_state_dict: dict | None = None,
                   optim_state_dict: dict | None = None, options: StateDictOptions | None = None):
    res = None
    if model_state_dict is not None:
        res = set_model_state_dict(model, model_state_dict, options=options)
    if optimizers is not None and optim_state_dict is not None:
        set_optimizer_state_dict(model, optimizers, optim_state_dict, options=options)
    return res


__all__: Iterable[str] = ["StateDictOptions", "get_model_state_dict", "get_optimizer_state_dict", "get_state_dict",
                          "set_model_state_dict", "set_optimizer_state_dict", "set_state_dict"]
