#!/usr/bin/env python3
"""Generate the README's MODELLED scaling section from the cost model (anx/cost.hpp).

usage: python tools/scaling_readme.py            # print the section
       python tools/scaling_readme.py --write    # replace it in README.md (between the markers)

tests/test_cost_model.py fails when README.md and this output differ, so the README's 1/2/4/8-GPU
tables are always the model's, never hand-edited numbers."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BEGIN, END = "<!-- scaling-model:begin -->\n", "<!-- scaling-model:end -->"
CONFIGS = [
    ("dp", 128, "local", "dp (the bench default): 128 images per GPU, weak scaling, outputs gathered to rank 0"),
    ("v4", 256, "root", "V4 (BASELINE config 3): 256 images in all from the host, strong scaling"),
    ("v5", 1024, "local", "V5 (BASELINE config 4): 1024 images in all, device-resident input, strong scaling"),
    ("v5", 1024, "root", "V5 with the reference's data flow (root scatters the batch every step)"),
]


def render() -> str:
    from anx.parallel import cost
    out = []
    for wl, batch, src, title in CONFIGS:
        c = cost.curve(wl, batch, input_source=src, mode="overlap" if wl == "v4" else "per_layer")
        out.append(f"**{title}** (modelled, not measured)\n\n{cost.table(c)}\n")
    p = cost.curve("dp", 128)["params"]
    out.append(f"Model inputs: single-GPU throughput vs images per launch {p['rate']} (measured); H2D "
               f"{p['h2d_gbps']} GB/s per GPU (measured); root ingest slowdown {p['ingest_slowdown']} per 155 MB received "
               f"per step (measured, tools/probe_ingest.py; dp rank 0 sheds that share); xGMI {p['xgmi_gbps']} GB/s per link and direction and host memory "
               f"{p['host_gbps']} GB/s (assumed). `python -m anx plan --model dp|v4|v5` prints the per-term "
               f"breakdown.\n")
    return "\n".join(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--write", action="store_true")
    a = ap.parse_args()
    sec = render()
    if not a.write:
        print(sec)
        return
    path = os.path.join(ROOT, "README.md")
    with open(path) as f:
        text = f.read()
    i, j = text.index(BEGIN) + len(BEGIN), text.index(END)
    with open(path, "w") as f:
        f.write(text[:i] + sec + text[j:])


if __name__ == "__main__":
    main()
