#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd database (kernel trace) as markdown.

    python tools/prof_summary.py gpurun_out/<tag>/prof/<name>_results.db [--top 25] [--title T]
"""
import argparse
import glob
import sqlite3


def summarize(db_path, top=25, title=None, after_last=None, last_ms=None):
    db = sqlite3.connect(db_path)
    cur = db.cursor()
    procs = cur.execute("select pid, command from processes").fetchall()
    t0 = 0
    if after_last:
        # steady state only: dispatches after the last kernel matching the pattern (e.g. the
        # MIOpen find-mode reference kernels that run during warmup)
        row = cur.execute("select max(end) from kernels where name like ?", (f"%{after_last}%",)).fetchone()
        t0 = row[0] or 0
    if last_ms:
        # steady state only: the final `last_ms` of the trace (the timed steps, after the
        # warmup's library tuning and per-layer A/B selection)
        row = cur.execute("select max(end) from kernels").fetchone()
        t0 = max(t0, (row[0] or 0) - int(last_ms * 1e6))
    total_n, total_ns = cur.execute("select count(*), sum(duration) from kernels where start > ?", (t0,)).fetchone()
    span = cur.execute("select min(start), max(end) from kernels where start > ?", (t0,)).fetchone()
    tot = total_ns or 1
    rows = cur.execute("select name, count(*), sum(duration), avg(duration), 100.0 * sum(duration) / ? from kernels "
                       "where start > ? group by name order by sum(duration) desc limit ?", (tot, t0, top)).fetchall()
    rows = [(n, c, t / 1e3, a / 1e3, pct) for n, c, t, a, pct in rows]
    out = [f"# {title or 'rocprofv3 kernel summary'}", "",
           f"source: `{db_path}` (rocprofv3 --kernel-trace --stats)"
           + (f"; steady state after the last `{after_last}` dispatch" if after_last else "")
           + (f"; the last {last_ms:g} ms of the trace only" if last_ms else ""), ""]
    for pid, cmd in procs:
        out.append(f"* process {pid}: `{cmd[:200]}`")
    out += ["", f"* kernels dispatched: {total_n}", f"* summed kernel time: {total_ns / 1e6:.2f} ms",
            f"* first-to-last dispatch span: {(span[1] - span[0]) / 1e6:.2f} ms" if span[0] else "", "",
            "| # | kernel | calls | total ms | avg us | % |", "|---|---|---|---|---|---|"]
    for i, (name, calls, tot, avg, pct) in enumerate(rows):
        short = name if len(name) < 110 else name[:107] + "..."
        short = short.replace("|", "\\|")
        out.append(f"| {i + 1} | `{short}` | {calls} | {tot / 1e3:.3f} | {avg:.1f} | {pct:.1f} |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("db", nargs="+")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default=None)
    ap.add_argument("-o", "--out", default=None)
    ap.add_argument("--after-last", default=None, help="only dispatches after the last kernel matching this")
    ap.add_argument("--last-ms", type=float, default=None, help="only dispatches in the trace's last N ms")
    a = ap.parse_args()
    paths = [p for g in a.db for p in glob.glob(g, recursive=True)]
    text = "\n".join(summarize(p, a.top, a.title, a.after_last, a.last_ms) for p in paths)
    if a.out:
        open(a.out, "w").write(text)
    else:
        print(text)
