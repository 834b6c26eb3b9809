#!/usr/bin/env python3
"""Run-log warehouse and analytics CLI (the reference's `log_analysis.py` + analysis notebook,
SURVEY §2.8 A1-A4), on sqlite (duckdb is not available here) + pandas + matplotlib.

    log_analysis.py ingest --root DIR [--db FILE]     # walk DIR, parse every run record (SHA1-dedup)
    log_analysis.py query "SELECT ..."                 # ad-hoc SQL over the `runs` table
    log_analysis.py stats                              # mean / sd / ci95 / min per (source, version, np, batch)
    log_analysis.py speedup [--baseline v1]            # S = T(base, np1) / T, E = S / np  (+ self-relative)
    log_analysis.py plot speedup|efficiency|runtime --out FILE.png
    log_analysis.py export --fmt csv|parquet --out FILE

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
def ingest(root: str = typer.Option(".", help="directory to walk"), db: str = DEFAULT_DB):
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


if __name__ == "__main__":
    app()
