"""Self-verification of a multi-rank data-parallel run (bench.py ``--workload dp`` at N > 1).

The first real 8-GPU run of the pipeline happens on a node the builder cannot reach, so the run has to
prove itself in its own JSON:

* :func:`rank_identity` — who ran: the communicator's world size, every rank's device ordinal, PCI
  location / UUID and host, whether they are distinct devices, and the node's peer-access matrix
  (``hipDeviceCanAccessPeer``). The reference's ranks all silently shared GPU 0 (no
  ``cudaSetDevice`` anywhere); here a shared device is visible in the record.
* :func:`verify_gather` — that the gather moved the right bytes: every rank hashes the output it
  computed in the last step (an exact integer checksum of the fp32 bits), rank 0 hashes what landed in
  each rank's slot of ``y_global``, and the two must agree bit for bit. Each rank also checks two of its
  own images against the fp64 PyTorch oracle. The reference's only correctness signal was a size
  warning after its Gatherv (final_project/v2_mpi_only/2.2_scatter_halo/src/main.cpp:266-273).
* :func:`calibrate_root_batch` — rank 0 also receives the whole gather, which costs it compute; the
  cost model prices that share from a one-GPU probe (``dp_root_batch``), this measures it: per-rank
  lane compute spans are all-gathered while rank 0 receives, and the root's share is rescaled so its
  span matches the peers' mean.
* :class:`FirstCollectiveWatchdog` — a bounded wait for the first collectives with a rank-tagged error,
  instead of the backend's multi-minute default.
* :class:`SecondaryDeadline` — a bounded wait for everything after the headline measurement: the
  headline line is printed even if a secondary program hangs.
"""
from __future__ import annotations

import json
import os
import socket
import sys
import threading

import torch
import torch.distributed as dist


def _gather_obj(obj, world: int) -> list:
    if world == 1 or not dist.is_initialized():
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def rank_identity(device: torch.device) -> dict:
    """Collective. Every rank's device identity, gathered (the same dict on every rank)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    me = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "host": socket.gethostname(),
          "device": None, "pci": None, "uuid": None, "name": None}
    if device.type == "cuda":
        p = torch.cuda.get_device_properties(device)
        me["device"] = device.index
        me["name"] = p.name
        bus = getattr(p, "pci_bus_id", None)
        if bus is not None:
            me["pci"] = "%04x:%02x:%02x" % (getattr(p, "pci_domain_id", 0) or 0, bus, getattr(p, "pci_device_id", 0) or 0)
        uuid = getattr(p, "uuid", None)
        me["uuid"] = str(uuid) if uuid is not None else None
    ranks = _gather_obj(me, world)
    keys = [(r["host"], r["uuid"] or r["pci"] or r["device"]) for r in ranks]
    out = {"world_size": world, "backend": dist.get_backend() if dist.is_initialized() else None, "ranks": ranks,
           "distinct_devices": len(set(keys)) == len(keys) if device.type == "cuda" else None}
    if device.type == "cuda":
        n = torch.cuda.device_count()
        out["visible_devices"] = n
        out["peer_access"] = [[1 if i == j else int(torch.cuda.can_device_access_peer(i, j)) for j in range(n)]
                              for i in range(n)]
    return out


def tensor_crc(t: torch.Tensor) -> int:
    """Exact checksum of a float32 tensor's bits: sum_i bits_i * (i mod 65521 + 1) in wrapping int64
    (integer addition, so every reduction order gives the same value)."""
    v = t.detach().contiguous().view(torch.int32).reshape(-1).to(torch.int64)
    w = torch.arange(v.numel(), device=v.device, dtype=torch.int64) % 65521 + 1
    return int((v * w).sum().item())


def verify_gather(pipe, oracle=None, corrupt_rank: int | None = None) -> dict:
    """Collective; call after ``pipe.drain()`` and a device sync, with the last step's outputs in place.

    Rank r hashes the rows it computed (``pipe.y``); rank 0 hashes slot r of ``y_global`` (root: its
    own ``root_batch`` rows; peers: ``batch_per_rank``). ``oracle(x_img, y_img) -> max rel err`` checks
    two local images (first and last) on every rank. ``corrupt_rank`` (tests) flips that rank's
    reported checksum, as a corrupted transfer would look."""
    world = pipe.world
    n_mine = pipe.y.shape[0]
    crc = tensor_crc(pipe.y[:n_mine])
    if corrupt_rank is not None and pipe.rank == corrupt_rank:
        crc ^= 1
    err = None
    if oracle is not None and pipe.x_used is not None and n_mine > 0:
        err = max(oracle(pipe.x_used[i:i + 1], pipe.y[i:i + 1]) for i in sorted({0, n_mine - 1}))
    mine = {"rank": pipe.rank, "images": n_mine, "crc": crc, "oracle_max_rel_err": err}
    allr = _gather_obj(mine, world)
    out = {"gather_verified": None, "per_rank": allr}
    if pipe.rank == 0 and pipe.y_global is not None:
        ok = []
        for r in allr:
            got = tensor_crc(pipe.y_global[r["rank"], :r["images"]])
            ok.append(got == r["crc"])
            r["crc_at_root"] = got
        out["gather_verified"] = all(ok)
        out["mismatched_ranks"] = [r["rank"] for r, g in zip(allr, ok) if not g]
    errs = [r["oracle_max_rel_err"] for r in allr if r["oracle_max_rel_err"] is not None]
    out["oracle_max_rel_err"] = max(errs) if errs else None
    return out


def _even_clamp(v: float, lo: int, hi: int) -> int:
    return max(lo, min(hi, 2 * int(round(v / 2))))


def calibrate_root_batch(pipe, step, sync, min_root: int, rounds: int = 2, steps: int = 8) -> dict:
    """Collective. Measure every rank's mean lane compute span while the pipeline runs (rank 0
    receiving the gather) and rescale rank 0's share to the peers' mean: rb' = rb * mean(peer spans) /
    root span, even, within [min_root, batch_per_rank]. Runs ``rounds`` x (``steps`` timed steps); every
    rank applies the same rb (all-gathered from rank 0)."""
    world = pipe.world
    B = pipe.cfg.batch_per_rank
    hist = []
    for _ in range(rounds):
        pipe.drain()
        sync()
        pipe.timing = True
        for _ in range(steps):
            step()
        pipe.drain()
        sync()
        pipe.timing = False
        span = pipe.lane_span_ms()
        spans = _gather_obj(span, world)
        rb = pipe.root_batch
        peer = sum(spans[1:]) / max(1, len(spans) - 1)
        new = _even_clamp(rb * peer / spans[0], min_root, B) if spans[0] > 0 and peer > 0 else rb
        new = _gather_obj(new, world)[0]  # rank 0's decision everywhere
        hist.append({"root_batch": rb, "span_ms": [round(s, 4) for s in spans], "next": new})
        if new == rb:
            break
        pipe.drain()
        sync()
        pipe.set_root_batch(new)
    return {"calibrated_root_batch": pipe.root_batch, "calibration": hist}


class FirstCollectiveWatchdog:
    """``with FirstCollectiveWatchdog(rank, seconds, what):`` — if the block (process-group setup and
    the first collectives) has not finished after ``seconds``, print a rank-tagged error and end the
    process with exit code 124 (a peer that never joined, a wrong master address, a dead device), rather
    than wait out the backend's default timeout."""

    def __init__(self, rank: int, seconds: float, what: str = "first collective"):
        self.rank, self.seconds, self.what = rank, seconds, what
        self._done = threading.Event()

    def _watch(self):
        if not self._done.wait(self.seconds):
            sys.stderr.write(f"[bench rank {self.rank}] {self.what} did not complete within {self.seconds:.0f} s "
                             f"(a peer missing or stuck): exiting\n")
            sys.stderr.flush()
            os._exit(124)

    def __enter__(self):
        if self.seconds > 0:
            threading.Thread(target=self._watch, daemon=True).start()
        return self

    def __exit__(self, *exc):
        self._done.set()
        return False


class SecondaryDeadline:
    """The headline's safety net for the work bench.py does after measuring it (batch-1 probes, the native
    V4 / V5 programs of BASELINE configs 3-4, the bf16 extension, the closing barrier). Those programs'
    device transports (RCCL point-to-point, peer IPC) meet real multi-GPU hardware for the first time in the
    driver's N > 1 runs; a call that hangs there would otherwise take the already-measured headline with it.
    If ``done()`` has not been called after ``seconds``, rank 0 prints ``rec`` (the headline record, built
    before any secondary ran) with ``secondary_deadline: {seconds, pending_stage}`` unless the full record
    was already printed, and every rank exits 0. ``emit(rec)`` prints the record exactly once.
    ``hang="<stage>:<rank>"`` (tests) makes that rank block at that stage, as a hung transport would."""

    def __init__(self, rank: int, seconds: float, rec: dict | None, hang: str | None = None):
        self.rank, self.seconds, self.rec = rank, seconds, rec
        self._hang = hang.rsplit(":", 1) if hang else None
        self._stage = "start"
        self._printed = False
        self._lock = threading.Lock()
        self._done = threading.Event()
        if seconds > 0:
            threading.Thread(target=self._watch, daemon=True).start()

    def stage(self, name: str) -> None:
        self._stage = name
        if self._hang and self._hang[0] == name and int(self._hang[1]) == self.rank:
            threading.Event().wait()  # never set: only the deadline ends this rank

    def emit(self, rec: dict) -> None:
        with self._lock:
            if not self._printed:
                self._printed = True
                print(json.dumps(rec), flush=True)

    def done(self) -> None:
        self._done.set()

    def _watch(self):
        if self._done.wait(self.seconds):
            return
        sys.stderr.write(f"[bench rank {self.rank}] secondary records still running after {self.seconds:.0f} s "
                         f"(stage: {self._stage}): headline kept, exiting 0\n")
        sys.stderr.flush()
        if self.rank == 0 and self.rec is not None:
            with self._lock:
                if not self._printed:
                    self._printed = True
                    r = dict(self.rec)
                    r["secondary_deadline"] = {"seconds": self.seconds, "pending_stage": self._stage}
                    sys.stdout.write(json.dumps(r) + "\n")
                    sys.stdout.flush()
        os._exit(0)
