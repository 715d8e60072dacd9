#!/usr/bin/env python3
"""HBM traffic per launch of the benchmark's dominant kernel from rocprofv3 PMC counters.

Follows MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
  * FETCH_SIZE and WRITE_SIZE are collected in SEPARATE --pmc passes (TCC slots: FETCH_SIZE costs
    3, WRITE_SIZE 2 -- they do not fit one pass), with --kernel-trace only (no sys/runtime trace);
  * both are reported in KiB -> x1024;
  * gfx950: FETCH_SIZE reads exactly 1/2 of the bytes of a wide coalesced streaming read
    (16 B/lane) -> x2; WRITE_SIZE is exact for 16-B streaming stores (our stores are 4-B
    per-row scalars: uncalibrated, they are <0.01 % of the bytes here).
Writes profiles/<tag>_pmc_traffic.json, which bench.py reads for roofline.traffic.

usage: python tools/pmc_traffic.py --tag r01 [-- bench args]
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter, outdir, bench_args):
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "-d", outdir, "-o", "run", "--output-format", "csv", "--",
           sys.executable, os.path.join(REPO, "bench.py")] + bench_args
    subprocess.run(cmd, check=True, cwd=REPO, stdout=subprocess.DEVNULL)
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    assert files, f"no counter csv under {outdir}"
    per_kernel = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            val = float(row.get("Counter_Value", 0) or 0)
            per_kernel.setdefault(name, []).append(val)
    return per_kernel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("bench_args", nargs="*")
    a = ap.parse_args()
    bench_args = a.bench_args or ["--steps", "5", "--warmup", "2", "--no-cpu", "--no-sweep", "--no-gpt2"]
    out = os.path.join(REPO, "gpurun_out", f"pmc_{a.tag}")
    fetch = run_pass("FETCH_SIZE", out + "_fetch", bench_args)
    write = run_pass("WRITE_SIZE", out + "_write", bench_args)
    kernels = {}
    for name, vals in fetch.items():
        if "copyBuffer" in name:
            continue
        f_kib = sum(vals) / len(vals)
        w_vals = write.get(name, [0.0])
        w_kib = sum(w_vals) / len(w_vals)
        kernels[name] = {
            "dispatches": len(vals),
            "FETCH_SIZE_KiB_mean": f_kib,
            "WRITE_SIZE_KiB_mean": w_kib,
            "hbm_bytes_per_launch": int(f_kib * 1024 * 2 + w_kib * 1024),
            "correction": "bytes = 2 * FETCH_SIZE * 1024 (gfx950 half-count of wide streaming reads) + WRITE_SIZE * 1024",
        }
    res = {"bench_args": bench_args, "kernels": kernels}
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    for d in ("profiles", "gpurun_out"):  # gpurun_out/ is what a GPU-box run hands back
        os.makedirs(os.path.join(REPO, d), exist_ok=True)
        json.dump(res, open(os.path.join(REPO, d, f"{a.tag}_pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
