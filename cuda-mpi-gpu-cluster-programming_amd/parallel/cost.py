"""Modelled multi-GPU scaling: Python face of the native cost model (csrc/src/cost.cpp, anx/cost.hpp).

One GPU is all the test boxes give, so the 2/4/8-GPU curve of every BASELINE configuration is
MODELLED from measured single-GPU inputs (engine throughput vs images per launch, the host link's
H2D rate, the root's compute slowdown while it ingests a gather) plus assumed link rates (xGMI per
link and direction), and every result carries ``"measured": false``. The reference derives its
speedup / efficiency from measurements afterwards: S = T(V1, np=1) / T, E = S / np
(/root/reference/log_analysis.py:212-222); here S and E are the model's.

The same model picks the runtimes' default row split (``pick_row_ways``): the V4 and V5 runtimes call
it natively, so what ``python -m anx plan --model`` prints is what they run.

Overrides: ``"name=value;..."`` over the defaults (``xgmi_gbps``, ``h2d_gbps``, ``d2h_gbps``,
``host_gbps``, ``ingest_slowdown`` (per 155 MB received per step), ``dp_root_shed``, ``stage1_share``, ``split_penalty``, ``phase_latency_ms``,
``v4_fill``, ``v5_chunks``; ``rate=IMAGES:IMG_PER_S,...`` replaces the throughput table).
"""
from __future__ import annotations

import ctypes as C
import json

from .. import _native as nat

WORKLOADS = {"dp": 0, "v4": 1, "v5": 2}
SOURCES = {"local": 0, "root": 1}
MODES = {"overlap": 0, "per_layer": 1}
NPS = (1, 2, 4, 8)


def _ov(overrides) -> bytes:
    if isinstance(overrides, dict):
        overrides = ";".join(f"{k}={v}" for k, v in overrides.items())
    return (overrides or "").encode()


def curve(workload: str, batch: int, nps=NPS, row_ways: int = -1, input_source: str = "local",
          mode: str = "per_layer", overrides=None) -> dict:
    """Modelled step time, throughput, speedup, efficiency and bound for each N in ``nps``."""
    arr = (C.c_int * len(nps))(*nps)
    buf = C.create_string_buffer(1 << 16)
    nat.call("anx_cost_curve", WORKLOADS[workload], arr, len(nps), batch, row_ways, SOURCES[input_source],
             MODES[mode], _ov(overrides), buf, len(buf))
    return json.loads(buf.value.decode())


def step(workload: str, np_: int, batch: int, row_ways: int = -1, input_source: str = "local",
         mode: str = "per_layer", overrides=None) -> dict:
    """One modelled step (bytes per phase, per-term milliseconds, bound)."""
    buf = C.create_string_buffer(1 << 13)
    nat.call("anx_cost_step", WORKLOADS[workload], np_, batch, row_ways, SOURCES[input_source], MODES[mode],
             _ov(overrides), buf, len(buf))
    return json.loads(buf.value.decode())


def pick_row_ways(workload: str, np_: int, batch: int, input_source: str = "local", mode: str = "per_layer",
                  overrides=None) -> int:
    """The row split the runtimes default to: the lowest modelled step over the divisors of np."""
    r = C.c_int()
    nat.call("anx_cost_pick_row_ways", WORKLOADS[workload], np_, batch, SOURCES[input_source], MODES[mode],
             _ov(overrides), C.byref(r))
    return r.value


def dp_root_batch(np_: int, batch: int, overrides=None) -> int:
    """dp: the images rank 0 computes per step while each peer computes ``batch`` -- the root's share
    shrunk by its modelled slowdown while it receives the gather (ingest_slowdown x bytes / 155 MB)."""
    r = C.c_int()
    nat.call("anx_cost_dp_root_batch", np_, batch, _ov(overrides), C.byref(r))
    return r.value


def table(c: dict) -> str:
    """Markdown table of a curve (the README's scaling section is generated from these); dp curves add
    the images rank 0 computes per step (its shed share)."""
    dp = c.get("workload") == "dp"
    head = "| N | row ways | " + ("rank-0 images | " if dp else "") + "step ms | images/s | speedup | efficiency | bound |"
    lines = [head, "|---:|---:|" + ("---:|" if dp else "") + "---:|---:|---:|---:|---|"]
    for i, n in enumerate(c["N"]):
        root = f"{c['root_batch'][i]} | " if dp else ""
        lines.append(f"| {n} | {c['row_ways'][i]} | {root}{c['step_ms'][i]:.3f} | {c['images_per_s'][i]:,.0f} | "
                     f"{c['speedup'][i]:.2f} | {c['efficiency'][i]:.2f} | {c['bound'][i]} |")
    return "\n".join(lines)
