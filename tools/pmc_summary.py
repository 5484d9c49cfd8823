"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs) into per-launch HBM-side
bytes per kernel, with the gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
FETCH_SIZE (KiB) counts half the bytes of wide coalesced reads -> x2; WRITE_SIZE (KiB) is exact.
Usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json>"""
import csv
import json
import sys


def per_kernel(path, counter):
    agg = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        agg.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(fetch_dir, write_dir, out):
    f = per_kernel(fetch_dir + "/run_counter_collection.csv", "FETCH_SIZE")
    w = per_kernel(write_dir + "/run_counter_collection.csv", "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        if "scvx::" not in k:
            continue
        short = k.split("(")[0].replace("void ", "")
        fb = 2.0 * 1024 * f.get(k, 0.0)
        wb = 1024 * w.get(k, 0.0)
        res[short] = {"fetch_bytes_corrected": fb, "write_bytes": wb, "traffic_bytes": fb + wb,
                      "raw_FETCH_SIZE_KiB": f.get(k), "raw_WRITE_SIZE_KiB": w.get(k)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
