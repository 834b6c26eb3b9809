#!/usr/bin/env python3
"""Run-log warehouse and analytics CLI (the reference's `log_analysis.py` + analysis notebook,
SURVEY §2.8 A1-A4), on sqlite (duckdb is not available here) + pandas + matplotlib.

    log_analysis.py ingest --root DIR [--db FILE]     # walk DIR, parse every run record (SHA1-dedup)
    log_analysis.py query "SELECT ..."                 # ad-hoc SQL over the `runs` table
    log_analysis.py stats                              # mean / sd / ci95 / min per (source, version, np, batch)
    log_analysis.py speedup [--baseline v1]            # S = T(base, np1) / T, E = S / np  (+ self-relative)
    log_analysis.py plot speedup|efficiency|runtime --out FILE.png
    log_analysis.py export --fmt csv|parquet --out FILE
    log_analysis.py report --out REPORT.md [--ref-root DIR]   # the notebook's synthesis views

Understood record formats (everything becomes one row: source, version, np, batch, time_ms, ...):
  * `ANX_JSON {...}` lines from `anx` / `python -m anx run` (time = warm_ms if present, else cold_ms)
  * bench.py JSON lines ({"metric": ..., "ms_per_step": ...})
  * harness CSV (scripts/common.sh 20-column schema — the reference's schema,
    scripts/0_run_final_project.sh:41) — rows with ExecutionTime_ms
  * the reference's own run logs: `... completed in <ms> ms` / `Execution Time: <ms> ms` lines in
    run_<version>_np<N>.log files (so its published numbers can be ingested as the baseline)
"""
from __future__ import annotations

import csv
import hashlib
import json
import math
import os
import re
import sqlite3
import sys

import typer

app = typer.Typer(add_completion=False, help=__doc__.split("\n")[0])
DEFAULT_DB = os.path.join(".warehouse", "anx_runs.sqlite")

SCHEMA = """
CREATE TABLE IF NOT EXISTS runs (
  id INTEGER PRIMARY KEY, sha1 TEXT UNIQUE, source TEXT, path TEXT, version TEXT, np INTEGER,
  batch INTEGER, time_ms REAL, cold_ms REAL, images_per_s REAL, shape TEXT, checksum TEXT,
  device TEXT, extra TEXT
);
"""
_TIME_RE = re.compile(r"(?:completed in|Execution Time:|ExecutionTime_ms[=:])\s*(-?[0-9.]+)\s*(?:ms)?")
_RUNLOG_RE = re.compile(r"run_(v[0-9.]+|v2_2\.[12]_\w+|v[0-9]_[\w.]+?)_np(\d+)\.log$")


def _db(path: str) -> sqlite3.Connection:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    c = sqlite3.connect(path)
    c.executescript(SCHEMA)
    return c


def _norm_version(v: str) -> str:
    v = v.lower()
    for pat, out in (("2.1", "v2.1"), ("2_1", "v2.1"), ("broadcast", "v2.1"), ("2.2", "v2.2"), ("2_2", "v2.2"),
                     ("scatter", "v2.2")):
        if pat in v:
            return out
    m = re.match(r"v?(\d)", v)
    return f"v{m.group(1)}" if m else v


def parse_file(path: str):
    """Yield row dicts from one file."""
    name = os.path.basename(path)
    try:
        text = open(path, errors="replace").read()
    except OSError:
        return
    if name.endswith(".csv"):
        rows = list(csv.DictReader(text.splitlines()))
        if rows and "ExecutionTime_ms" in rows[0]:
            for r in rows:
                try:
                    t = float(r["ExecutionTime_ms"])
                except (TypeError, ValueError):
                    continue
                yield dict(source="harness-csv", version=_norm_version(r.get("ProjectVariant", "")),
                           np=int(r.get("NumProcesses") or 1), batch=1, time_ms=t, cold_ms=t,
                           shape=r.get("OutputShape", ""), checksum="", device=r.get("MachineID", ""))
        return
    found = False
    for line in text.splitlines():
        line = line.strip()
        if line.startswith("ANX_JSON "):
            d = json.loads(line[9:])
            t = d.get("warm_ms") or d.get("cold_ms")
            found = True
            yield dict(source="anx-native" if d.get("native") else "anx-python", version=d["version"], np=d["np"],
                       batch=d["batch"], time_ms=t, cold_ms=d.get("cold_ms"), images_per_s=d.get("images_per_s"),
                       shape="x".join(map(str, d.get("shape", []))), checksum=str(d.get("checksum", "")),
                       device=d.get("device", ""), extra=json.dumps(d.get("phases_warm") or d.get("phases_cold")))
        elif line.startswith("{") and '"metric"' in line:
            try:
                d = json.loads(line)
            except json.JSONDecodeError:
                continue
            found = True
            yield dict(source="bench", version="bench-" + d["config"].get("parallelism", ""), np=d["n_gpus"],
                       batch=d["config"].get("global_batch", 0), time_ms=d["ms_per_step"], cold_ms=None,
                       images_per_s=d["value"], shape="", checksum="", device="MI355X", extra=json.dumps(d["config"]))
    if not found:
        m = _RUNLOG_RE.search(name)
        if m:
            t = _TIME_RE.search(text)
            if t:
                yield dict(source="reference-log", version=_norm_version(m.group(1)), np=int(m.group(2)), batch=1,
                           time_ms=float(t.group(1)), cold_ms=float(t.group(1)), shape="", checksum="",
                           device=os.path.basename(os.path.dirname(path)))


@app.command()
def ingest(root: str = typer.Option(".", help="directory to walk"), db: str = DEFAULT_DB,
           tag: str = typer.Option("", help="prefix for the source label (e.g. 'reference' for its tree)")):
    """Walk ROOT and load every run record (dedup by SHA1 of path+record)."""
    c = _db(db)
    n = 0
    for dp, _, files in os.walk(root):
        if ".warehouse" in dp or "/.git" in dp:
            continue
        for f in files:
            if not f.endswith((".log", ".csv", ".jsonl", ".json", ".out")):
                continue
            p = os.path.join(dp, f)
            for row in parse_file(p):
                if tag and not row["source"].startswith(tag):
                    row["source"] = f"{tag}-{row['source']}"
                key = hashlib.sha1((p + json.dumps(row, sort_keys=True)).encode()).hexdigest()
                row = {**dict(images_per_s=None, extra=""), **row}
                try:
                    c.execute("INSERT INTO runs (sha1, source, path, version, np, batch, time_ms, cold_ms, images_per_s,"
                              " shape, checksum, device, extra) VALUES (?,?,?,?,?,?,?,?,?,?,?,?,?)",
                              (key, row["source"], p, row["version"], row["np"], row["batch"], row["time_ms"],
                               row["cold_ms"], row["images_per_s"], row["shape"], row["checksum"], row["device"],
                               row["extra"]))
                    n += 1
                except sqlite3.IntegrityError:
                    pass
    c.commit()
    typer.echo(f"ingested {n} new rows into {db}")


@app.command()
def query(sql: str, db: str = DEFAULT_DB):
    """Run SQL against the warehouse and print the result."""
    import pandas as pd
    typer.echo(pd.read_sql_query(sql, _db(db)).to_string(index=False))


def _stats_df(db):
    import pandas as pd
    df = pd.read_sql_query("SELECT source, version, np, batch, time_ms FROM runs WHERE time_ms > 0", _db(db))
    g = df.groupby(["source", "version", "np", "batch"])["time_ms"]
    out = g.agg(n="count", mean="mean", sd="std", min="min").reset_index()
    out["ci95"] = 1.96 * out["sd"].fillna(0) / out["n"].map(math.sqrt)  # reference: log_analysis.py:176-198
    return out


@app.command()
def stats(db: str = DEFAULT_DB):
    """Mean / sd / 95% CI / best per (source, version, np, batch)."""
    typer.echo(_stats_df(db).to_string(index=False, float_format=lambda v: f"{v:.3f}"))


def _speedup_df(db, baseline: str):
    s = _stats_df(db)
    rows = []
    for (src, b), grp in s.groupby(["source", "batch"]):
        base = grp[(grp.version == baseline) & (grp.np == 1)]
        for _, r in grp.iterrows():
            own = grp[(grp.version == r.version) & (grp.np == 1)]
            t1 = float(own["min"].iloc[0]) if len(own) else float("nan")
            tb = float(base["min"].iloc[0]) if len(base) else float("nan")
            rows.append(dict(source=src, batch=b, version=r.version, np=r.np, best_ms=r["min"],
                             speedup_vs_base=tb / r["min"], speedup_self=t1 / r["min"],
                             efficiency_self=t1 / r["min"] / r.np))
    import pandas as pd
    return pd.DataFrame(rows)


@app.command()
def speedup(baseline: str = "v1", db: str = DEFAULT_DB):
    """Speedup vs BASELINE at np=1 (log_analysis.py:212-222) and self-relative (analysis.md:222-250)."""
    typer.echo(_speedup_df(db, baseline).to_string(index=False, float_format=lambda v: f"{v:.3f}"))


@app.command()
def plot(kind: str = typer.Argument(..., help="speedup | efficiency | runtime"), out: str = "plot.png",
         source: str = "", db: str = DEFAULT_DB):
    """Line plot per version over np (runtime = best ms)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    df = _speedup_df(db, "v1")
    if source:
        df = df[df.source == source]
    col = {"speedup": "speedup_self", "efficiency": "efficiency_self", "runtime": "best_ms"}[kind]
    fig, ax = plt.subplots(figsize=(6, 4))
    for (src, ver, b), g in df.groupby(["source", "version", "batch"]):
        g = g.sort_values("np")
        ax.plot(g.np, g[col], marker="o", label=f"{ver} ({src}, b={b})")
    ax.set_xlabel("ranks / GPUs")
    ax.set_ylabel(kind)
    if kind == "runtime":
        ax.set_yscale("log")
    ax.legend(fontsize=6)
    ax.grid(alpha=0.3)
    fig.tight_layout()
    fig.savefig(out, dpi=120)
    typer.echo(f"wrote {out}")


@app.command()
def export(fmt: str = "csv", out: str = "runs.csv", db: str = DEFAULT_DB):
    """Export the raw runs table (csv | parquet)."""
    import pandas as pd
    df = pd.read_sql_query("SELECT * FROM runs", _db(db))
    if fmt == "parquet":
        df.to_parquet(out)
    else:
        df.to_csv(out, index=False)
    typer.echo(f"wrote {len(df)} rows to {out}")


# Source files that make up each version's own code path (non-blank, non-comment lines counted),
# ours and the reference's (its notebook's version_loc_map, analysis.md Cell 19).
OUR_VERSION_SOURCES = {
    "v1": ["csrc/src/cpu/ref_layers.cpp", "csrc/src/cpu/blocks_cpu.cpp"],
    "v2.1": ["csrc/src/cpu/ref_layers.cpp", "csrc/src/cpu/blocks_cpu.cpp", "csrc/src/comm/host_comm.cpp"],
    "v2.2": ["csrc/src/cpu/ref_layers.cpp", "csrc/src/cpu/blocks_cpu.cpp", "csrc/src/comm/host_comm.cpp",
             "csrc/src/plan.cpp"],
    "v3": ["csrc/src/engine.cpp", "csrc/src/hip/conv_mfma.hip", "csrc/src/hip/winograd.hip",
           "csrc/src/hip/conv1_wino.hip", "csrc/src/hip/pool_lrn.hip"],
    "v4": ["csrc/src/engine.cpp", "csrc/src/hip/conv_mfma.hip", "csrc/src/hip/winograd.hip",
           "csrc/src/hip/conv1_wino.hip", "csrc/src/hip/pool_lrn.hip", "csrc/src/comm/host_comm.cpp",
           "csrc/src/plan.cpp"],
    "v5": ["csrc/src/engine.cpp", "csrc/src/hip/conv_mfma.hip", "csrc/src/hip/winograd.hip",
           "csrc/src/hip/conv1_wino.hip", "csrc/src/hip/pool_lrn.hip", "csrc/src/plan.cpp",
           "csrc/src/runtime/schedule.cpp", "csrc/src/comm/device_comm.cpp"],
}
REF_VERSION_DIRS = {
    "v1": ["final_project/v1_serial"], "v2.1": ["final_project/v2_mpi_only/2.1_broadcast_all"],
    "v2.2": ["final_project/v2_mpi_only/2.2_scatter_halo"], "v3": ["final_project/v3_cuda_only"],
    "v4": ["final_project/v4_mpi_cuda"], "v5": ["final_project/v5_cuda_aware_mpi"],
}
_SRC_EXT = (".cpp", ".cu", ".hip", ".hpp", ".h", ".c", ".inl", ".cuh")


def _loc(path: str) -> int:
    n, block = 0, False
    try:
        for line in open(path, errors="replace"):
            t = line.strip()
            if block:
                block = "*/" not in t
                continue
            if not t or t.startswith("//"):
                continue
            if t.startswith("/*"):
                block = "*/" not in t
                continue
            n += 1
    except OSError:
        return 0
    return n


def _loc_tree(root: str, dirs: list[str]) -> int:
    total = 0
    for d in dirs:
        for dp, _, files in os.walk(os.path.join(root, d)):
            total += sum(_loc(os.path.join(dp, f)) for f in files if f.endswith(_SRC_EXT))
    return total


@app.command()
def report(out: str = "report.md", plot_out: str = "", ref_root: str = "", repo_root: str = ".",
           db: str = DEFAULT_DB):
    """The notebook's synthesis views (analysis.md Cells 17-19) as one markdown report: ours vs the
    reference per version, scaling with the Karp-Flatt serial fraction, and code size vs speedup."""
    import pandas as pd
    sp = _speedup_df(db, "v1")
    lines = ["# Run-log synthesis", "", f"warehouse: `{db}`, {len(sp)} (source, batch, version, np) groups", ""]
    # 1. ours vs the reference's logged runs, per version and np (batch 1: the reference's config)
    ours = sp[(sp.source == "anx-native") & (sp.batch == 1)]
    ref = sp[sp.source.str.startswith("reference")]  # its logs, and its CSVs ingested with --tag reference
    rows = []
    for _, r in ours.iterrows():
        rr = ref[(ref.version == r.version) & (ref.np == r.np)]
        if len(rr):
            t_ref = float(rr.best_ms.min())
            rows.append(dict(version=r.version, np=int(r.np), ours_ms=r.best_ms, reference_best_ms=t_ref,
                             speedup_over_reference=t_ref / r.best_ms))
    lines += ["## Ours vs the reference's own logged runs (batch 1, best of each)", ""]
    if rows:
        lines += [pd.DataFrame(rows).to_markdown(index=False, floatfmt=".3f"), ""]
    else:
        lines += ["(no overlapping version / np between the two sources)", ""]
    # 2. scaling: self-relative speedup, efficiency, Karp-Flatt experimentally determined serial fraction
    lines += ["## Scaling (self-relative) and the Karp-Flatt serial fraction e = (1/S - 1/p) / (1 - 1/p)", ""]
    sc = sp[sp.np > 1].copy()
    sc["karp_flatt"] = (1.0 / sc.speedup_self - 1.0 / sc.np) / (1.0 - 1.0 / sc.np)
    if len(sc):
        lines += [sc[["source", "batch", "version", "np", "best_ms", "speedup_self", "efficiency_self", "karp_flatt"]]
                  .sort_values(["source", "batch", "version", "np"]).to_markdown(index=False, floatfmt=".3f"), ""]
    # 3. code size vs speed (the notebook's LOC x performance synthesis)
    loc = []
    for v, files in OUR_VERSION_SOURCES.items():
        row = dict(version=v, ours_loc=sum(_loc(os.path.join(repo_root, f)) for f in files))
        if ref_root:
            row["reference_loc"] = _loc_tree(ref_root, REF_VERSION_DIRS[v])
        for b in sorted(ours.batch.unique()) if len(ours) else []:
            g = sp[(sp.source == "anx-native") & (sp.batch == b) & (sp.version == v) & (sp.np == 1)]
            row[f"speedup_vs_v1_b{b}"] = float(g.speedup_vs_base.iloc[0]) if len(g) else float("nan")
        loc.append(row)
    ldf = pd.DataFrame(loc)
    lines += ["## Code size per version vs speed (np = 1)", "",
              "Lines of code of each version's own path (non-blank, non-comment; ours: the files each "
              "version runs, shared kernels counted in every version that uses them).", "",
              ldf.to_markdown(index=False, floatfmt=".2f"), ""]
    spcols = [c for c in ldf.columns if c.startswith("speedup_vs_v1_b")]
    if spcols and ldf[spcols[-1]].notna().sum() >= 3:
        from scipy.stats import pearsonr
        ok = ldf[ldf[spcols[-1]].notna()]
        r, pval = pearsonr(ok.ours_loc, ok[spcols[-1]].map(math.log10))
        lines += [f"Pearson r(ours LOC, log10 speedup at {spcols[-1][-4:]}) = {r:.2f} (p = {pval:.2g}, "
                  f"{len(ok)} versions): the larger paths are the device versions (V3-V5, MFMA kernels, "
                  f"Winograd, runtime), which are also the fast ones.", ""]
        if plot_out:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt
            fig, ax = plt.subplots(figsize=(6, 4))
            ax.scatter(ok.ours_loc, ok[spcols[-1]], label="anx (MI355X)")
            for _, q in ok.iterrows():
                ax.annotate(q.version, (q.ours_loc, q[spcols[-1]]), fontsize=8)
            ax.set_xlabel("lines of code of the version's path")
            ax.set_ylabel(f"speedup vs V1 ({spcols[-1][-4:]})")
            ax.set_yscale("log")
            ax.grid(alpha=0.3)
            fig.tight_layout()
            fig.savefig(plot_out, dpi=120)
            lines += [f"![speedup vs LOC]({os.path.basename(plot_out)})", ""]
    with open(out, "w") as f:
        f.write("\n".join(lines))
    typer.echo(f"wrote {out}")


if __name__ == "__main__":
    app()
