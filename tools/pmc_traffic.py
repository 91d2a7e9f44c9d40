#!/usr/bin/env python3
"""HBM bytes per collect from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KiB), merged into profiles/hbm_traffic.json.

    python tools/pmc_traffic.py --fetch <dir>/kb_counter_collection.csv --write <dir>/kb_counter_collection.csv \
        --kernel collect_kernel --workload north_star --docs 1000000000 --bytes 10000000000 --merge profiles/hbm_traffic.json

A collect may be several kernels (config 3: the hot-slot pass, the cold-list count and the slab reduce; config 4: the HLL
phases and gathers): --kernel takes a comma list of name substrings and --collects the number of collects the run made,
so the figure is the bytes of every matching dispatch divided by the collects.  Without --collects, the dispatches of
the first kernel name count as the collects (one dispatch per collect).

FETCH_SIZE is doubled: on gfx950 it reports half the bytes of 16-byte-per-lane streaming reads
(MI355X_MICROARCH.md, "HBM [CDNA4]").  WRITE_SIZE is taken as reported.  The output entry is keyed by (workload, docs,
shards); bench.py reads the entry matching its run.
"""
import argparse
import csv
import json
import os


def totals(path, kernels, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    tot, n_first, names = 0.0, 0, set()
    for r in rows:
        for i, k in enumerate(kernels):
            if k in r["Kernel_Name"]:
                tot += float(r["Counter_Value"])
                names.add(r["Kernel_Name"].split("(")[0])
                n_first += 1 if i == 0 else 0
                break
    if not names:
        raise SystemExit(f"no {counter} rows for {kernels} in {path}")
    return tot, n_first, sorted(names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="collect_kernel", help="comma list of kernel-name substrings of one collect")
    ap.add_argument("--collects", type=int, default=0, help="collects in each pass (0: dispatches of the first kernel)")
    ap.add_argument("--workload", default="north_star")
    ap.add_argument("--docs", type=int, default=1_000_000_000)
    ap.add_argument("--shards", type=int, default=1, help="shards of the bench run (bench --shards; 1 = one per GPU)")
    ap.add_argument("--bytes", type=int, required=True, help="algorithmic bytes per collect (the layout's, bench bytes_per_doc)")
    ap.add_argument("--merge", default="", help="hbm_traffic.json to add / replace the entry in (else print it)")
    a = ap.parse_args()
    kernels = [k for k in a.kernel.split(",") if k]
    f, nf, names = totals(a.fetch, kernels, "FETCH_SIZE")
    w, nw, _ = totals(a.write, kernels, "WRITE_SIZE")
    cf = a.collects or nf
    cw = a.collects or nw
    hbm = int(2 * f * 1024 / cf + w * 1024 / cw)
    entry = {
        "workload": a.workload, "docs": a.docs, "shards": a.shards, "kernels": names,
        "fetch_size_kib_per_collect": f / cf, "write_size_kib_per_collect": w / cw, "collects": [cf, cw],
        "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": a.bytes, "traffic_over_algorithmic": hbm / a.bytes,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes with --kernel-trace; FETCH_SIZE "
                  "doubled for 16-B/lane streaming reads per MI355X_MICROARCH.md 'HBM [CDNA4]'; WRITE_SIZE as reported; "
                  "every kernel of one collect summed",
    }
    if not a.merge:
        print(json.dumps(entry, indent=1))
        return
    doc = {"entries": []}
    if os.path.exists(a.merge):
        with open(a.merge) as fh:
            old = json.load(fh)
        doc = old if "entries" in old else {"entries": []}
    doc["entries"] = [e for e in doc["entries"]
                      if (e["workload"], e["docs"], e.get("shards", 1)) != (a.workload, a.docs, a.shards)] + [entry]
    with open(a.merge, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(entry))


if __name__ == "__main__":
    main()
