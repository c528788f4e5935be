#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes
for the hot kernel, corrected as MI355X_MICROARCH.md §HBM prescribes:
  * FETCH_SIZE / WRITE_SIZE are in KiB (x1024);
  * gfx950 FETCH_SIZE reports exactly half of a wide coalesced streaming read
    (16 B/lane global_load_dwordx4, which is this kernel's access) -> x2;
  * WRITE_SIZE is exact for 16 B/lane streaming stores.
Usage: pmc_traffic.py FETCH_CSV WRITE_CSV KEY ALGO_BYTES_PER_LAUNCH [OUT_JSON]
Merges {KEY: {...}} into OUT_JSON (default profiles/pmc_traffic.json)."""
import csv
import json
import os
import statistics
import sys


def per_launch(path, counter, kernel_substr="k_fwd8x8_quant"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel_substr in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return statistics.median(vals), len(vals)


def main():
    fetch_csv, write_csv, key, algo = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4])
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json")
    f_kib, nf = per_launch(fetch_csv, "FETCH_SIZE")
    w_kib, nw = per_launch(write_csv, "WRITE_SIZE")
    read_b = f_kib * 1024 * 2
    write_b = w_kib * 1024
    entry = {"fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib, "launches": [nf, nw],
             "read_bytes_corrected": read_b, "write_bytes": write_b,
             "hbm_bytes_per_launch": read_b + write_b, "algorithmic_bytes_per_launch": algo,
             "traffic_over_algorithmic": (read_b + write_b) / algo,
             "correction": "FETCH_SIZE x1024 x2 (gfx950 half-count of 16B/lane streaming reads), WRITE_SIZE x1024"}
    d = json.load(open(out)) if os.path.exists(out) else {}
    d[key] = entry
    json.dump(d, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: entry}, indent=1))


if __name__ == "__main__":
    main()
