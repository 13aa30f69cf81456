"""Worker process entry point (one per GPU), started by the launcher.

Initialises the process group over the launcher's TCPStore (RCCL "nccl" backend with GPUs,
gloo on CPU - Ray TorchConfig semantics, timeout 1800 s), installs the session, runs the
user's `train_loop_per_worker(config)`, waits for queued async checkpoint commits, and
publishes success/failure to the control plane.
"""
from __future__ import annotations

import datetime
import inspect
import os
import signal
import sys
import threading
import time
import traceback

import cloudpickle
import torch
import torch.distributed as dist
from torch.distributed import PrefixStore, TCPStore


def _heartbeat(store, key, stop):
    while not stop.is_set():
        try:
            store.set(key, str(time.time()))
        except Exception:
            return
        stop.wait(2.0)


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ["LOCAL_RANK"])
    attempt = int(os.environ.get("RTDC_ATTEMPT", "0"))
    with open(os.environ["RTDC_PAYLOAD"], "rb") as f:
        payload = cloudpickle.load(f)
    store = TCPStore("127.0.0.1", int(os.environ["RTDC_STORE_PORT"]), is_master=False,
                     timeout=datetime.timedelta(seconds=payload["timeout_s"]))
    stop = threading.Event()
    hb = threading.Thread(target=_heartbeat, args=(store, f"a{attempt}/hb/{rank}", stop), daemon=True)
    hb.start()
    from . import session as S
    from .checkpoint import Checkpoint

    sess = None
    try:
        use_gpu = payload["use_gpu"]
        backend = payload.get("backend") or ("nccl" if use_gpu else "gloo")
        if use_gpu:
            torch.cuda.set_device(local)
        pg_store = PrefixStore(f"pg{attempt}", store)
        kw = {}
        if use_gpu and backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, store=pg_store, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=payload["timeout_s"]), **kw)
        ctx = S.TrainContext(world, rank, local, world, 0, payload["experiment_name"], payload["trial_dir"],
                             payload["storage_path"], os.path.basename(payload["trial_dir"]), attempt,
                             torch_config=payload.get("torch_config"),
                             checkpoint_config=payload["checkpoint_config"])
        from ..checkpoint import torchsave

        cc = payload["checkpoint_config"]
        if hasattr(cc, "ring_slots"):  # size the native engine's pinned ring from the typed config
            torchsave.configure_engine(cc.ring_slots, cc.ring_slot_mb, cc.writer_threads)
        resume = payload.get("resume_checkpoint")
        sess = S._Session(ctx, store, payload["checkpoint_config"], Checkpoint(resume) if resume else None)
        fail_at = os.environ.get("RTDC_FAIL_AT_REPORT")
        if fail_at and attempt == 0:
            k, _, r = fail_at.partition(":")
            if not r or int(r) == rank:
                orig = sess.report

                def report_then_die(*a, **kw2):
                    orig(*a, **kw2)
                    if sess.n_reports >= int(k):
                        os.kill(os.getpid(), signal.SIGKILL)

                sess.report = report_then_die
        S._set_session(sess)
        fn = payload["fn"]
        cfg = payload["config"]
        if len(inspect.signature(fn).parameters) == 0:
            fn()
        else:
            fn(cfg)
        sess.close()
        store.add(f"a{attempt}/ndone", 1)
        code = 0
    except BaseException:
        tb = traceback.format_exc()
        sys.stderr.write(tb)
        try:
            store.set(f"a{attempt}/error/{rank}", tb)
            store.add(f"a{attempt}/nerrors", 1)
        except Exception:
            pass
        code = 1
    finally:
        stop.set()
        try:
            if dist.is_initialized():
                if code == 0:
                    dist.destroy_process_group()
        except Exception:
            pass
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(code)


if __name__ == "__main__":
    main()
