"""A minimal Metaflow-compatible flow runner for the two reference flows.

Provides what R/train_flow.py and R/eval_flow.py use, with the same CLI:
  python train_flow.py [--environment=...] run [--epochs 3 --batch_size 32 --learning_rate 1e-3
                                                --from-run F/R --from-task F/R/S/T]
  python train_flow.py argo-workflows create | trigger      (local deployment registry)
  python eval_flow.py  run [--from-run ... --from-task ... --from-namespace ... --batch_size 512]

* `FlowSpec`, `@step`, `Parameter` (flag names/defaults as declared; the string "null" is
  passed through like Metaflow so flows can treat it as unset), `self.next(...)` including
  `num_parallel=N` gangs (the control task runs the body - metaflow-ray semantics - and the
  N-1 worker tasks carry no artifacts, so the reference `join` step works unchanged);
* `current` (flow/run/step/task ids, `ray_storage_path`, `card`, `trigger`, `parallel`);
* decorators: `@retry(times)`, `@metaflow_ray`, `@gpu_profile(interval)`, `@card(type, id)`,
  `@schedule(cron)`, `@trigger_on_finish(flow)`; `@kubernetes/@pypi/@conda/@resources` are
  accepted and ignored (one node);
* artifacts persisted to the local run registry (flow/registry.py), client `Run`/`Task`.
A finished run fires the deployed flows that declared `@trigger_on_finish` on it.
"""
from __future__ import annotations

import argparse
import inspect
import json
import os
import subprocess
import sys
import time
import traceback

from . import registry
from .cards import CardRegistry

# ------------------------------------------------------------------------------ current
class _Parallel:
    def __init__(self, num_nodes=1, node_index=0, main_ip="127.0.0.1"):
        self.num_nodes, self.node_index, self.main_ip = num_nodes, node_index, main_ip


class _Trigger:
    def __init__(self, run_pathspec: str | None):
        self._ps = run_pathspec

    @property
    def run(self):
        if not self._ps:
            raise AttributeError("this run was not triggered by another flow")
        return registry.Run(self._ps)


class _Current:
    def __init__(self):
        self._reset()

    def _reset(self):
        self.flow_name = None
        self.run_id = None
        self.step_name = None
        self.task_id = None
        self.retry_count = 0
        self.ray_storage_path = None
        self.card = CardRegistry()
        self._trigger = None
        self.parallel = _Parallel()
        self.is_running_flow = False
        self.namespace = "user:" + os.environ.get("USER", "local")
        self.username = os.environ.get("USER", "local")

    @property
    def pathspec(self):
        return f"{self.flow_name}/{self.run_id}/{self.step_name}/{self.task_id}"

    @property
    def trigger(self):
        if self._trigger is None:
            raise AttributeError("current.trigger is unavailable: the run was not event-triggered")
        return self._trigger


current = _Current()


# ------------------------------------------------------------------------------ decorators
def _deco(name, **kw):
    def wrap(f):
        decos = getattr(f, "_rtdc_decos", {})
        decos[name] = kw
        f._rtdc_decos = decos
        return f

    return wrap


def step(f):
    f._rtdc_step = True
    if not hasattr(f, "_rtdc_decos"):
        f._rtdc_decos = {}
    return f


def retry(f=None, *, times: int = 3, minutes_between_retries: int = 0):
    if f is not None and callable(f):
        return _deco("retry", times=3, minutes_between_retries=0)(f)
    return _deco("retry", times=times, minutes_between_retries=minutes_between_retries)


def metaflow_ray(f=None, *, all_nodes_started_timeout: int = 300, **kw):
    if f is not None and callable(f):
        return _deco("metaflow_ray", all_nodes_started_timeout=300)(f)
    return _deco("metaflow_ray", all_nodes_started_timeout=all_nodes_started_timeout)


def gpu_profile(f=None, *, interval: float = 1.0, **kw):
    if f is not None and callable(f):
        return _deco("gpu_profile", interval=1.0)(f)
    return _deco("gpu_profile", interval=interval)


def card(f=None, *, type: str = "default", id: str | None = None, **kw):  # noqa: A002
    if f is not None and callable(f):
        return _deco("card", type="default", id="default")(f)
    return _deco("card", type=type, id=id or "default")


def _noop_factory(name):
    def deco(f=None, **kw):
        if f is not None and callable(f):
            return f
        return lambda g: g

    deco.__name__ = name
    return deco


kubernetes = _noop_factory("kubernetes")
pypi = _noop_factory("pypi")
conda = _noop_factory("conda")
resources = _noop_factory("resources")
environment = _noop_factory("environment")


def schedule(cls=None, *, cron: str | None = None, hourly=False, daily=False, weekly=False):
    def wrap(c):
        c._rtdc_schedule = cron or ("0 * * * *" if hourly else "0 0 * * *" if daily else "0 0 * * 0" if weekly else None)
        return c

    return wrap(cls) if cls is not None else wrap


def trigger_on_finish(cls=None, *, flow: str | None = None, flows=None):
    def wrap(c):
        c._rtdc_trigger_on_finish = [flow] if flow else list(flows or [])
        return c

    return wrap(cls) if cls is not None else wrap


# ------------------------------------------------------------------------------ parameters
class Parameter:
    def __init__(self, name: str, default=None, help: str | None = None, type=None, required=False):  # noqa: A002
        self.name, self.default, self.help, self.required = name, default, help, required
        self.type = type or (builtins_type(default) if default is not None else str)

    def parse(self, raw):
        if raw is None:
            return self.default
        if self.type is bool:
            return str(raw).lower() in ("1", "true", "yes")
        try:
            return self.type(raw)
        except (TypeError, ValueError):
            return raw


def builtins_type(v):
    return {bool: bool, int: int, float: float}.get(type(v), str)


class _Inputs(list):
    pass


class _TaskView:
    """Artifacts of one finished task (the `inputs` of a join step)."""

    def __init__(self, artifacts: dict):
        self.__dict__.update(artifacts)


# ------------------------------------------------------------------------------ FlowSpec
class FlowSpec:
    _rtdc_schedule = None
    _rtdc_trigger_on_finish: list = []

    def __init__(self, use_cli: bool = True):
        self._next = None
        self._num_parallel = None
        if use_cli:
            sys.exit(self._cli(sys.argv[1:]))

    # -- graph API ---------------------------------------------------------------------
    def next(self, *steps, num_parallel: int | None = None, foreach: str | None = None):
        if len(steps) != 1:
            raise NotImplementedError("branching is not supported; use a linear graph / num_parallel")
        self._next = steps[0].__name__
        self._num_parallel = num_parallel

    @classmethod
    def _params(cls):
        out = {}
        for klass in reversed(cls.__mro__):
            for k, v in vars(klass).items():
                if isinstance(v, Parameter):
                    out[k] = v
        return out

    @classmethod
    def _flow_name(cls):
        return cls.__name__

    def _artifacts(self) -> dict:
        skip = set(self._params())
        return {k: v for k, v in self.__dict__.items() if not k.startswith("_") and k not in skip}

    # -- CLI ---------------------------------------------------------------------------
    def _cli(self, argv) -> int:
        top = argparse.ArgumentParser(prog=os.path.basename(sys.argv[0]), add_help=True)
        top.add_argument("--environment", default=None)
        top.add_argument("--with", dest="with_", action="append", default=[])
        top.add_argument("--datastore", default=None)
        top.add_argument("--metadata", default=None)
        top.add_argument("--quiet", action="store_true")
        top.add_argument("--no-pylint", action="store_true")
        top.add_argument("command", nargs="?", default="run")
        top.add_argument("rest", nargs=argparse.REMAINDER)
        a = top.parse_args(argv)
        cmd = a.command
        if cmd in ("run", "evaluate"):  # README's `evaluate` (R/README.md:24) means `run`
            return self._cmd_run(a.rest)
        if cmd == "argo-workflows":
            sub = a.rest[0] if a.rest else "create"
            return self._cmd_deploy(sub, a.rest[1:])
        if cmd == "show":
            print(self._describe())
            return 0
        print(f"unknown command {cmd!r}; supported: run, show, argo-workflows create|trigger", file=sys.stderr)
        return 2

    def _param_parser(self):
        p = argparse.ArgumentParser(prog="run")
        for attr, prm in self._params().items():
            p.add_argument(f"--{prm.name}", dest=attr, default=None, help=prm.help)
        p.add_argument("--tag", action="append", default=[])
        p.add_argument("--max-workers", default=None)
        p.add_argument("--rtdc-trigger-run", dest="_trigger_run", default=None, help=argparse.SUPPRESS)
        return p

    def _describe(self):
        steps = [n for n, f in inspect.getmembers(type(self), inspect.isfunction) if getattr(f, "_rtdc_step", False)]
        return json.dumps({"flow": self._flow_name(), "steps": steps,
                           "parameters": {p.name: p.default for p in self._params().values()},
                           "schedule": self._rtdc_schedule, "trigger_on_finish": self._rtdc_trigger_on_finish})

    def _cmd_deploy(self, sub, rest) -> int:
        flow = self._flow_name()
        if sub == "create":
            registry.save_deployment(flow, {"file": os.path.abspath(sys.argv[0]), "schedule": self._rtdc_schedule,
                                            "trigger_on_finish": self._rtdc_trigger_on_finish})
            print(f"[rtdc] deployed {flow} (schedule={self._rtdc_schedule}, "
                  f"trigger_on_finish={self._rtdc_trigger_on_finish}) to {registry.home()}")
            return 0
        if sub == "trigger":
            deps = registry.load_deployments()
            if flow not in deps:
                print(f"{flow} is not deployed; run `argo-workflows create` first", file=sys.stderr)
                return 1
            return self._cmd_run(rest)
        if sub in ("delete", "remove"):
            deps = registry.load_deployments()
            deps.pop(flow, None)
            with open(os.path.join(registry.home(), "_deployments.json"), "w") as f:
                json.dump(deps, f)
            return 0
        print(f"unsupported: argo-workflows {sub}", file=sys.stderr)
        return 2

    # -- execution ---------------------------------------------------------------------
    def _cmd_run(self, rest) -> int:
        args = self._param_parser().parse_args(rest)
        flow = self._flow_name()
        for attr, prm in self._params().items():
            setattr(self, attr, prm.parse(getattr(args, attr)))
        run_id = registry.new_run_id(flow)
        current._reset()
        current.flow_name, current.run_id, current.is_running_flow = flow, run_id, True
        if args._trigger_run:
            current._trigger = _Trigger(args._trigger_run)
        params = {prm.name: getattr(self, attr) for attr, prm in self._params().items()}
        registry.write_run_meta(flow, run_id, status="running", params=params, started=time.time(),
                                triggered_by=args._trigger_run)
        print(f"[rtdc] {flow}/{run_id} starting (registry {registry.home()})", flush=True)
        ok = False
        try:
            self._execute(flow, run_id)
            ok = True
        except Exception:
            traceback.print_exc()
        registry.write_run_meta(flow, run_id, status="succeeded" if ok else "failed", finished=time.time())
        print(f"[rtdc] {flow}/{run_id} {'succeeded' if ok else 'FAILED'}", flush=True)
        if ok:
            self._fire_triggers(flow, run_id)
        return 0 if ok else 1

    def _execute(self, flow, run_id):
        cls = type(self)
        step_name = "start"
        inputs = None
        task_counter = 0
        while step_name is not None:
            fn = getattr(cls, step_name)
            decos = getattr(fn, "_rtdc_decos", {})
            n_par = self._num_parallel if (self._next == step_name and self._num_parallel) else 1
            self._next, self._num_parallel = None, None
            task_counter += 1
            task_id = str(task_counter)
            tries = decos.get("retry", {}).get("times", 0) + 1
            for attempt in range(tries):
                current.step_name, current.task_id, current.retry_count = step_name, task_id, attempt
                current.card = CardRegistry()
                current.parallel = _Parallel(num_nodes=n_par, node_index=0)
                tdir = registry.task_dir(flow, run_id, step_name, task_id)
                os.makedirs(tdir, exist_ok=True)
                if "metaflow_ray" in decos:
                    current.ray_storage_path = os.path.join(tdir, f"ray_storage_attempt{attempt}")
                    os.makedirs(current.ray_storage_path, exist_ok=True)
                else:
                    current.ray_storage_path = None
                if "card" in decos:
                    _ = current.card[decos["card"]["id"]]
                prof = None
                if "gpu_profile" in decos:
                    from ..utils.profiling import GpuProfiler

                    prof = GpuProfiler(decos["gpu_profile"].get("interval", 1.0), out_dir=tdir).start()
                try:
                    print(f"[rtdc] {flow}/{run_id}/{step_name}/{task_id} (attempt {attempt})", flush=True)
                    if inputs is not None and len(inspect.signature(fn).parameters) > 1:
                        fn(self, inputs)
                    else:
                        fn(self)
                    err = None
                except Exception as e:
                    err = e
                    traceback.print_exc()
                finally:
                    if prof is not None:
                        prof.stop()
                        current.card["gpu_profile"].extend(prof.card_components())
                for cid, c in current.card.items():
                    c.save(os.path.join(tdir, "cards"), f"{flow}/{run_id}/{step_name}/{task_id} - {cid}")
                if err is None:
                    break
                if attempt + 1 >= tries:
                    raise err
            registry.save_artifacts(tdir, self._artifacts())
            nxt = self._next
            if n_par > 1:
                # worker tasks of the gang (metaflow-ray: they host workers, no artifacts)
                for w in range(1, n_par):
                    task_counter += 1
                    os.makedirs(registry.task_dir(flow, run_id, step_name, str(task_counter)), exist_ok=True)
                inputs = _Inputs([_TaskView(self._artifacts())] + [_TaskView({}) for _ in range(n_par - 1)])
            elif nxt is not None and getattr(getattr(cls, nxt), "_rtdc_decos", None) is not None and \
                    len(inspect.signature(getattr(cls, nxt)).parameters) > 1:
                inputs = _Inputs([_TaskView(self._artifacts())])
            else:
                inputs = None
            if step_name == "end":
                break
            if nxt is None:
                raise RuntimeError(f"step {step_name} did not call self.next(...)")
            step_name = nxt

    def _fire_triggers(self, flow, run_id):
        for name, dep in registry.load_deployments().items():
            if flow in (dep.get("trigger_on_finish") or []) and os.path.exists(dep.get("file", "")):
                print(f"[rtdc] {flow}/{run_id} finished -> triggering deployed flow {name}", flush=True)
                env = dict(os.environ, RTDC_HOME=registry.home())
                subprocess.call([sys.executable, dep["file"], "run", "--rtdc-trigger-run", f"{flow}/{run_id}"], env=env)
