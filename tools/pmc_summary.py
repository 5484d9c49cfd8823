"""Summarise the rocprofv3 --pmc passes of tools/gpu_pmc.sh (one counter group per run) for one kernel.

HBM-side bytes per launch follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE (KiB)
counts half the bytes of wide coalesced reads on gfx950 -> x2; WRITE_SIZE (KiB) is exact.  SQ cycle
counters (SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_*) count quad-cycles (x4 = shader cycles); the
SQ_INSTS_* counters count wave-instructions.

usage: python tools/pmc_summary.py <gpurun_out/pmc_TAG> <out.json> [kernel-substring] [skip]
       (reads every <gpurun_out/pmc_TAG>_*/run_counter_collection.csv)
skip: drop each pass's first `skip` dispatches of the kernel from the per-launch averages (the PMC
command's warmup launch is a cold QP start; the bench's timed launches are warm-started, so skip=1
gives the timed region's per-launch figures); the all-launch traffic is kept as traffic_bytes_all."""
import collections
import csv
import glob
import json
import sys


def collect(prefix, kernel, skip=0):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for f in sorted(glob.glob(prefix + "_*/run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            key = (f, int(r["Dispatch_Id"]))
            per[r["Counter_Name"]][key] += float(r["Counter_Value"])
            names[r["Counter_Name"]] = r["Kernel_Name"]
    out = {}
    for c, v in per.items():
        keep = []
        for f in sorted({k[0] for k in v}):
            keep += sorted((k for k in v if k[0] == f), key=lambda k: k[1])[skip:]
        out[c] = sum(v[k] for k in keep) / max(len(keep), 1)
    return out, names


def main(prefix, out, kernel="qp_ipm_kernel<scvx::QPCfg<6, 3, 2, 8, 0, 0>", skip="0"):
    skip = int(skip)
    c, names = collect(prefix, kernel, skip)
    res = {"kernel": next(iter(names.values()), kernel).split("(")[0].replace("void ", ""),
           "source": prefix + "_*", "skipped_first_dispatches_per_pass": skip, "raw_per_launch": c}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fb, wb = 2.0 * 1024 * c["FETCH_SIZE"], 1024 * c["WRITE_SIZE"]
        res.update(fetch_bytes_corrected=fb, write_bytes=wb, traffic_bytes=fb + wb)
        if skip:
            ca, _ = collect(prefix, kernel, 0)
            res["traffic_bytes_all"] = 2.0 * 1024 * ca["FETCH_SIZE"] + 1024 * ca["WRITE_SIZE"]
    w = c.get("SQ_WAVES")
    if w and "SQ_WAVE_CYCLES" in c:
        cyc = 4 * c["SQ_WAVE_CYCLES"] / w
        d = {"wave_cycles": cyc}
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA"):
            if k in c:
                d[k.lower().replace("sq_", "") + "_frac"] = 4 * c[k] / w / cyc
        for k in ("SQ_INSTS_VALU", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                  "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU"):
            if k in c:
                d[k.lower().replace("sq_", "") + "_per_wave"] = c[k] / w
        if "SQ_INSTS_VALU_FMA_F64" in c:
            f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                               "SQ_INSTS_VALU_TRANS_F64"))
            d["f64_share_of_valu_insts"] = f64 / max(c.get("SQ_INSTS_VALU", 1.0), 1.0)
            d["issued_f64_flop_per_launch_64lanes"] = 64 * (2 * c["SQ_INSTS_VALU_FMA_F64"] + c.get("SQ_INSTS_VALU_ADD_F64", 0)
                                                             + c.get("SQ_INSTS_VALU_MUL_F64", 0))
        res["per_wave"] = d
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        res["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
