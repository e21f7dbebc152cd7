"""Turn rocprofv3 PMC passes into the bench's roofline.traffic figure.

Input : gpurun_out/pmc/p*/run_counter_collection.csv from tools/pmc.sh with
        separate passes "FETCH_SIZE" and "WRITE_SIZE" (they cannot share a pass
        on gfx950: TCC slots), and gpurun_out/pmc/trace/run_kernel_stats.csv.
Output: profiles/<round>_fwd_traffic.json

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports exactly half of the bytes of a wide coalesced
streaming read (16 B/lane global_load and buffer_load … lds alike), so
HBM bytes = 2·FETCH_SIZE·1024 + WRITE_SIZE·1024, per dispatch of the kernel.
"""
import csv, glob, json, os, statistics, sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pmc = sys.argv[1] if len(sys.argv) > 1 else os.path.join(root, "gpurun_out", "pmc")
rnd = sys.argv[2] if len(sys.argv) > 2 else "r01"
kern = sys.argv[3] if len(sys.argv) > 3 else "dense_fwd_w8q2_wide"
vals = {}
for f in glob.glob(os.path.join(pmc, "p*", "run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        if kern in row["Kernel_Name"] and row["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE"):
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
fetch = statistics.median(vals["FETCH_SIZE"]) * 1024
write = statistics.median(vals["WRITE_SIZE"]) * 1024
N, d, BH = 4096, 64, 64
alg = BH * (3 * N * d * 2 + N * d * 2 + 2 * N * 4)
out = {"workload": "configs[1]", "kernel": kern,
       "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
       "hbm_bytes_per_launch": 2 * fetch + write,
       "algorithmic_bytes_per_launch": alg,
       "ratio_to_algorithmic": (2 * fetch + write) / alg,
       "dispatches": len(vals["FETCH_SIZE"]),
       "note": "HBM bytes = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE half-count correction); "
               "algorithmic = Q,K,V read once + O written once + l,m (bf16 in/out, fp32 l,m)"}
path = os.path.join(root, "profiles", f"{rnd}_fwd_traffic.json")
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(out, indent=1))
