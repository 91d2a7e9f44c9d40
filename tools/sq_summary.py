#!/usr/bin/env python3
"""SQ counter summary of the collect kernel from rocprofv3 --pmc CSV passes (kb_counter_collection.csv per pass dir):
per-dispatch sums averaged over dispatches, merged over the passes, and the ratios DESIGN §5 / §9 quote.

    python tools/sq_summary.py --docs 1000000000 gpurun_out/<tag>/pmc_north_star_* > profiles/.../x_sq_counters.json
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="collect_kernel")
    ap.add_argument("--docs", type=float, required=True, help="docs per dispatch (the per-256-doc instruction counts)")
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    out, meta = {}, {}
    for d in a.dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            per = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                if a.kernel not in r["Kernel_Name"]:
                    continue
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                meta = {"kernel": r["Kernel_Name"].split("(")[0], "vgpr": r.get("VGPR_Count") or r.get("Arch_VGPR_Count"),
                        "sgpr": r.get("SGPR_Count"), "lds": r.get("LDS_Block_Size")}
            n = len(per)
            for dd in per.values():
                for k, v in dd.items():
                    out[k] = out.get(k, 0.0) + v / n
    w = out.get("SQ_WAVES", 0)
    r = {}
    if w:
        steps = a.docs / w / 256.0
        for k in ("VALU", "SALU", "LDS", "VMEM_RD"):
            if f"SQ_INSTS_{k}" in out:
                r[f"{k}_per_wave_per_256_docs"] = round(out[f"SQ_INSTS_{k}"] / w / steps, 1)
    wc = out.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if k in out:
                r[f"{k}/SQ_WAVE_CYCLES"] = round(out[k] / wc, 3)
    if out.get("SQ_LDS_IDX_ACTIVE"):
        r["SQ_LDS_BANK_CONFLICT/SQ_LDS_IDX_ACTIVE"] = round(out["SQ_LDS_BANK_CONFLICT"] / out["SQ_LDS_IDX_ACTIVE"], 3)
    print(json.dumps({"meta": meta, "ratios": r, "per_dispatch": out}, indent=1))


if __name__ == "__main__":
    main()
