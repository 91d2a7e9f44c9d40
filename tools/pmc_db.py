#!/usr/bin/env python3
"""Per-dispatch counter sums of a kernel from rocprofv3 rocpd databases (one per PMC pass), averaged over its dispatches.

    python tools/pmc_db.py --kernel collect_kernel gpurun_out/<tag>/p1/pass_results.db [...]
"""
import argparse
import collections
import json
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="collect_kernel")
    ap.add_argument("dbs", nargs="+")
    a = ap.parse_args()
    out, meta = {}, {}
    for path in a.dbs:
        db = sqlite3.connect(path)
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for disp, name, ctr, val, vg, sg, lds, dur in db.execute(
                "select dispatch_id, kernel_name, counter_name, value, vgpr_count, sgpr_count, lds_block_size, duration "
                "from counters_collection"):
            if a.kernel in name:
                per[disp][ctr] += val
                meta = {"kernel": name.split("(")[0][:120], "vgpr": vg, "sgpr": sg, "lds": lds}
                per[disp]["_dur_ns"] = dur
        n = len(per)
        if not n:
            continue
        for ctr in next(iter(per.values())):
            out[ctr] = sum(d[ctr] for d in per.values()) / n
        out["_dispatches_" + path.split("/")[-2]] = n
    print(json.dumps({"meta": meta, "per_dispatch": out}, indent=1))


if __name__ == "__main__":
    main()
