#!/usr/bin/env python3
"""HBM bytes per launch of the dominant kernel from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KiB).

    python tools/pmc_traffic.py --fetch <dir>/bench_counter_collection.csv --write <dir>/bench_counter_collection.csv \
        --kernel collect_kernel --workload north_star --docs 1000000000 --bytes 20000000000 > profiles/hbm_traffic.json

FETCH_SIZE is doubled: on gfx950 it reports half the bytes of 16-byte-per-lane streaming reads
(MI355X_MICROARCH.md, "HBM [CDNA4]").  WRITE_SIZE is taken as reported.
"""
import argparse
import csv
import json


def per_launch(path, kernel, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    return sum(vals) / len(vals), len(vals), [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]][0]["Kernel_Name"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="collect_kernel")
    ap.add_argument("--workload", default="north_star")
    ap.add_argument("--docs", type=int, default=1_000_000_000)
    ap.add_argument("--bytes", type=int, default=20_000_000_000, help="algorithmic bytes per launch")
    a = ap.parse_args()
    f, nf, name = per_launch(a.fetch, a.kernel, "FETCH_SIZE")
    w, nw, _ = per_launch(a.write, a.kernel, "WRITE_SIZE")
    hbm = int(2 * f * 1024 + w * 1024)
    print(json.dumps({
        "workload": a.workload, "docs": a.docs, "kernel": name,
        "fetch_size_kib_per_launch": f, "write_size_kib_per_launch": w, "dispatches": [nf, nw],
        "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": a.bytes, "traffic_over_algorithmic": hbm / a.bytes,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes with --kernel-trace; FETCH_SIZE "
                  "doubled for 16-B/lane streaming reads per MI355X_MICROARCH.md 'HBM [CDNA4]'; WRITE_SIZE as reported",
    }, indent=1))


if __name__ == "__main__":
    main()
