#!/usr/bin/env python3
"""Average PMC counters per dispatch of the kernels matching a substring, one rocprofv3 --pmc
pass per counter group (groups separated by ';'), kernel-trace only.

usage: python tools/pmc_kernel.py OUTDIR SUBSTR 'CTR CTR;CTR CTR' -- cmd args...
"""
import csv
import glob
import os
import subprocess
import sys


def main():
    out, sub, groups = sys.argv[1], sys.argv[2], sys.argv[3]
    cmd = sys.argv[sys.argv.index("--") + 1:]
    res = {}
    for gi, grp in enumerate(g.strip() for g in groups.split(";")):
        d = os.path.join(out, f"pass{gi}")
        subprocess.run(["timeout", "-s", "KILL", "90", "rocprofv3", "--pmc", *grp.split(), "--kernel-trace", "-d", d, "-o", "run",
                        "--output-format", "csv", "--"] + cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                name = row.get("Kernel_Name", "")
                if sub not in name:
                    continue
                key = (name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][-60:], row["Counter_Name"])
                res.setdefault(key, []).append(float(row.get("Counter_Value", 0) or 0))
    for (k, c), v in sorted(res.items()):
        print(f"{k:60s} {c:32s} n={len(v):4d} mean={sum(v) / len(v):.4g}")


if __name__ == "__main__":
    main()
