"""Summarise a rocprofv3 results .db (kernel trace, optional PMC) into text/JSON for profiles/."""
import json
import sqlite3
import sys
from pathlib import Path


def summarize(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
    out = {"kernels": [{"name": r[0][:160], "calls": r[1], "total_us": r[2], "avg_us": r[3], "pct": r[4]} for r in rows]}
    try:
        agg = {}
        for kname, cname, val in c.execute("select kernel_name, counter_name, value from counters_collection"):
            agg.setdefault((kname, cname), []).append(val or 0)
        if agg:
            out["pmc"] = [{"kernel": k[0][:120], "counter": k[1], "dispatches": len(v), "avg_per_dispatch": sum(v) / len(v)}
                          for k, v in sorted(agg.items())]
    except sqlite3.Error as e:
        out["pmc_error"] = str(e)
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1])
    txt = json.dumps(res, indent=1)
    if len(sys.argv) > 2:
        Path(sys.argv[2]).write_text(txt)
    print(txt[:4000])
