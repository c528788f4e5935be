#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes
for the hot kernel, corrected as MI355X_MICROARCH.md §HBM prescribes:
  * FETCH_SIZE / WRITE_SIZE are in KiB (x1024);
  * gfx950 FETCH_SIZE reports exactly half of a wide coalesced streaming read
    (16 B/lane global_load_dwordx4, which is this kernel's access) -> x2;
  * WRITE_SIZE is exact for 16 B/lane streaming stores.
Usage: pmc_traffic.py FETCH_CSV WRITE_CSV KEY ALGO_BYTES_PER_LAUNCH [OUT_JSON] [--kernels a,b,...]
Merges {KEY: {...}} into OUT_JSON (default profiles/pmc_traffic.json).
--kernels (config 4): the step is several launches -- per-launch medians of the
kernels whose names contain each substring, summed; reads are reported as the
64-B tally (FETCH_SIZE x1024 = TCC_EA0_RDREQ x 64 B, a lower bound: these
kernels read 8 B/lane row pieces, so the memory side sees a mix of 64-B and
128-B requests, the latter tallied at 64 B) with the all-128-B upper bound
beside it; writes exact."""
import csv
import json
import os
import statistics
import sys


def per_launch(path, counter, kernel_substr="k_fwd8x8_quant"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if kernel_substr in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return statistics.median(vals), len(vals)


def main_multi(fetch_csv, write_csv, key, algo, out, subs):
    f_kib = w_kib = 0.0
    per = {}
    for sub in subs:
        f, nf = per_launch(fetch_csv, "FETCH_SIZE", sub)
        w, nw = per_launch(write_csv, "WRITE_SIZE", sub)
        per[sub] = {"fetch_size_kib_raw": f, "write_size_kib_raw": w, "launches": [nf, nw]}
        f_kib += f
        w_kib += w
    read_lo, write_b = f_kib * 1024, w_kib * 1024
    entry = {"kernels": per, "read_bytes_64B_tally": read_lo, "read_bytes_if_all_128B": 2 * read_lo,
             "write_bytes": write_b, "hbm_bytes_per_launch": read_lo + write_b,
             "hbm_bytes_upper_bound": 2 * read_lo + write_b, "algorithmic_bytes_per_launch": algo,
             "traffic_over_algorithmic": (read_lo + write_b) / algo,
             "traffic_over_algorithmic_upper": (2 * read_lo + write_b) / algo,
             "correction": "per step = sum over the listed kernels; FETCH_SIZE x1024 as the 64-B request tally "
                           "(TCC_EA0_RDREQ x 64; lower bound for 8-B/lane row reads), WRITE_SIZE x1024"}
    d = json.load(open(out)) if os.path.exists(out) else {}
    d[key] = entry
    json.dump(d, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps({key: entry}, indent=1))


def main():
    args = [x for x in sys.argv[1:]]
    subs = None
    if "--kernels" in args:
        i = args.index("--kernels")
        subs = args[i + 1].split(",")
        del args[i:i + 2]
    fetch_csv, write_csv, key, algo = args[0], args[1], args[2], float(args[3])
    out = args[4] if len(args) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json")
    if subs:
        return main_multi(fetch_csv, write_csv, key, algo, out, subs)
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
