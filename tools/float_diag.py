"""Float diagnostics (GPU box): one request shape over the synthetic `price` column, the worst buckets by the GPU's
relative error against the oracle's exact sums, with the oracle's own error beside it.
    python3 tools/float_diag.py --docs 100000000 [--shape north_star|config2]
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "oracle"), os.path.join(os.path.dirname(HERE), "tests")]

import oracle as O  # noqa: E402
import elasticsearch_amd as ea  # noqa: E402
from elasticsearch_amd import AggregationBuilders as AB  # noqa: E402
from helpers import _rel, synthetic_columns  # noqa: E402


def walk(got, want, path, out):
    if isinstance(want, dict):
        if "_exact" in want:
            ex = want["_exact"]
            for k in ("sum", "avg"):
                if k in ex and isinstance(want.get(k), float):
                    out.append((_rel(got[k], ex[k]), _rel(want[k], ex[k]), path + "." + k, got[k], want[k], ex[k],
                                want.get("count")))
            return
        for k in want:
            if k in got:
                walk(got[k], want[k], path + "." + k, out)
    elif isinstance(want, list):
        for i, (g, w) in enumerate(zip(got, want)):
            walk(g, w, f"{path}[{i}]", out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=100_000_000)
    ap.add_argument("--shape", default="north_star")
    a = ap.parse_args()
    if a.shape == "north_star":
        fields = ("host", "@timestamp", "price")
        aggs = [AB.terms("hosts").field("host").size(10).subAggregation(
            AB.dateHistogram("per_hour").field("@timestamp").interval("1h").subAggregation(AB.stats("p").field("price")))]
    else:
        fields = ("@timestamp", "price")
        aggs = [AB.dateHistogram("h").field("@timestamp").interval("1h").subAggregation(AB.extendedStats("x").field("price")),
                AB.extendedStats("all").field("price")]
    cols = synthetic_columns(fields, a.docs)
    want = O.run([(cols, a.docs)], aggs, exact=True)["shards"][0]
    del cols
    eng = ea.Engine(0)
    seg = eng.synthetic_segment(a.docs, fields=fields)
    plan = eng.plan(aggs)
    plan.collect(seg)
    got = plan.build().to_dict()
    out = []
    walk(got, want, "", out)
    out.sort(reverse=True)
    print("values", len(out), "gpu == oracle:", sum(1 for o in out if o[3] == o[4]))
    for o in out[:8]:
        print("gpu_err %.3g oracle_err %.3g %s gpu %r oracle %r exact %r count %s" % o)


if __name__ == "__main__":
    main()
