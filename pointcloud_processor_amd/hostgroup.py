"""Host-side control plane of `bench.py --gpus N`: barriers, the max-over-ranks timing and the
RCCL id hand-off, with torch.distributed (gloo) kept OUT of the rank's process.

Why a helper process: a PyTorch wheel bundles its own HIP runtime, HSA runtime and RCCL under
the SONAMEs libpcp links (libamdhip64.so.7, librccl.so.1).  If torch is imported first, libpcp
silently runs on torch's copies; if libpcp is loaded first, importing torch maps a second HSA /
HIP stack into the process and the two clash at exit (double free in their destructors).  So
the process that runs libpcp never imports torch: each rank starts one helper child
(`python -m pointcloud_processor_amd.hostgroup`) that joins the gloo group from the same
environment (RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT -- torchrun's agent store included) and
executes the rank's control-plane calls, one JSON line per request over its stdin / stdout.
Nothing on the data path goes through it: the data-path collective is libpcp's own RCCL
communicator (pcp_comm_init_rank / pcp_raycast_fan_allreduce).
"""
from __future__ import annotations

import base64
import json
import os
import subprocess
import sys

import numpy as np


class HostGroup:
    """The rank's handle on its helper.  Same call order on every rank (collectives)."""

    def __init__(self):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        env = dict(os.environ)
        env.setdefault("MASTER_ADDR", "127.0.0.1")
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
        self._p = subprocess.Popen([sys.executable, "-u", "-m", "pointcloud_processor_amd.hostgroup"],
                                   stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=env,
                                   text=True, bufsize=1)
        self._call({"op": "hello"})

    def _call(self, req: dict):
        self._p.stdin.write(json.dumps(req) + "\n")
        self._p.stdin.flush()
        line = self._p.stdout.readline()
        if not line:
            raise RuntimeError(f"hostgroup helper of rank {self.rank} exited "
                               f"(code {self._p.poll()})")
        rep = json.loads(line)
        if "error" in rep:
            raise RuntimeError(f"hostgroup: {rep['error']}")
        return rep

    def barrier(self):
        self._call({"op": "barrier"})

    def allreduce(self, vec, op: str) -> np.ndarray:
        """Element-wise op ("sum" | "max" | "min") of a numeric vector over all ranks."""
        a = np.ascontiguousarray(vec)
        rep = self._call({"op": "allreduce", "red": op, "dtype": a.dtype.str,
                          "shape": list(a.shape), "data": base64.b64encode(a.tobytes()).decode()})
        return np.frombuffer(base64.b64decode(rep["data"]), a.dtype).reshape(a.shape).copy()

    def allreduce_np(self, vec, op: str) -> np.ndarray:   # pointcloud_processor_amd.dist
        return self.allreduce(vec, op)

    def broadcast_bytes(self, data: bytes | None, src: int = 0) -> bytes:
        rep = self._call({"op": "broadcast", "src": src,
                          "data": base64.b64encode(data or b"").decode()})
        return base64.b64decode(rep["data"])

    def close(self):
        if self._p.poll() is None:
            try:
                self._call({"op": "exit"})
            except (RuntimeError, OSError, ValueError):
                pass
            try:
                self._p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                self._p.kill()
                self._p.wait()


def _serve():
    """The helper: torch.distributed over gloo from the inherited environment."""
    out = os.fdopen(os.dup(1), "w")   # the protocol channel; stray prints go to stderr
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    import datetime

    # a rank that dies leaves the others' helpers in a collective: bounded, not gloo's 30 min
    dist.init_process_group(backend="gloo", timeout=datetime.timedelta(seconds=600))
    ops = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}
    try:
        for line in sys.stdin:
            req = json.loads(line)
            op = req["op"]
            try:
                if op == "hello":
                    rep = {"rank": dist.get_rank(), "world": dist.get_world_size()}
                elif op == "barrier":
                    dist.barrier()
                    rep = {}
                elif op == "allreduce":
                    a = np.frombuffer(base64.b64decode(req["data"]),
                                      np.dtype(req["dtype"])).reshape(req["shape"]).copy()
                    t = torch.from_numpy(a)
                    dist.all_reduce(t, op=ops[req["red"]])
                    rep = {"data": base64.b64encode(t.numpy().tobytes()).decode()}
                elif op == "broadcast":
                    obj = [base64.b64decode(req["data"])]
                    dist.broadcast_object_list(obj, src=int(req["src"]))
                    rep = {"data": base64.b64encode(obj[0]).decode()}
                elif op == "exit":
                    out.write("{}\n")
                    out.flush()
                    break
                else:
                    rep = {"error": f"unknown op {op}"}
            except Exception as e:   # the rank raises it; the group is then unusable
                rep = {"error": f"{type(e).__name__}: {e}"}
            out.write(json.dumps(rep) + "\n")
            out.flush()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    _serve()
