#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc passes (GN occupancy / fp64 mix, SVO HBM traffic).

usage: tools/pmc_kernels.py RUN_DIR OUT_JSON
RUN_DIR holds the sub-directories of tools/gpu_pmc.sh (gn_occ, gn_f64, svo_f, svo_w), each with a
run_counter_collection.csv.

Derived values (per dispatch, averaged over the dispatches of a kernel):
  * waves_per_cu  = SQ_WAVES / 256 CUs (the grid's own width: how many waves one launch gives a CU);
  * mean_resident_waves_per_cu = 4 * SQ_WAVE_CYCLES (quad-cycles, MI355X_MICROARCH.md) /
    (duration x 2.4 GHz x 256 CUs), against the 32 waves a CU holds (8 per SIMD).  The duration
    is the dispatch's own timestamps in the PMC run (kernels are serialised there);
  * valu_busy = SQ_ACTIVE_INST_VALU (quad-cycles) x 4 / (duration x 2.4 GHz x 256 CUs x 4 SIMDs);
  * fp64 lane-ops from SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 (wave instructions x 64 lanes, FMA = 2)
    and the rate they give over the kernel-trace duration against the MI355X fp64 vector peak
    (78.6 TFLOP/s, vendor specification; the guides do not list it);
  * HBM traffic = FETCH_SIZE x 2 (MI355X_MICROARCH.md gfx950 correction for 16-byte streaming
    reads; other widths uncalibrated) + WRITE_SIZE, in bytes per dispatch.
"""
from __future__ import annotations

import collections
import csv
import json
import os
import re
import sys

CUS, CLK_GHZ, FP64_PEAK_TFLOPS = 256, 2.4, 78.6


def short(name: str) -> str:
    base = name.replace("(anonymous namespace)::", "").split("(")[0]
    base = re.sub(r"<.*>", "", base)
    return base.split("::")[-1].strip()


def load(path):
    """{kernel: {dispatch: {counter: value, '_dur_ns': d}}}"""
    out = collections.defaultdict(dict)
    f = os.path.join(path, "run_counter_collection.csv")
    if not os.path.exists(f):
        return out
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        d = out[k].setdefault(int(r["Dispatch_Id"]), {"_dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                      "_vgpr": int(r["VGPR_Count"]), "_lds": int(r["LDS_Block_Size"]),
                                                      "_wg": int(r["Workgroup_Size"]), "_grid": int(r["Grid_Size"])})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def mean(ds, key):
    v = [d[key] for d in ds.values() if key in d]
    return sum(v) / len(v) if v else None


def main():
    run, out = sys.argv[1], sys.argv[2]
    occ, f64 = load(os.path.join(run, "gn_occ")), load(os.path.join(run, "gn_f64"))
    sf, sw = load(os.path.join(run, "svo_f")), load(os.path.join(run, "svo_w"))
    sq = load(os.path.join(run, "svo_sq"))
    res = {"source": f"rocprofv3 --pmc passes of tools/gpu_pmc.sh ({os.path.basename(run.rstrip('/'))})",
           "cus": CUS, "clock_ghz": CLK_GHZ, "gn": {}, "svo": {},
           # the library the passes ran (viso_version "src:"), when given
           "src": os.environ.get("SRC_HASH", "")}
    for k in ("direct_level_kernel", "lk_align_kernel", "pyr_down_sk_kernel"):
        if k not in occ:
            continue
        ds = occ[k]
        dur = mean(ds, "_dur_ns")
        cyc = dur * CLK_GHZ
        e = {"dispatches": len(ds), "pmc_duration_us": round(dur / 1e3, 2),
             "vgpr": int(mean(ds, "_vgpr")), "lds_bytes": int(mean(ds, "_lds")),
             "workgroup": int(mean(ds, "_wg")), "grid_threads": round(mean(ds, "_grid")),
             "waves": round(mean(ds, "SQ_WAVES"), 1),
             "waves_per_cu": round(mean(ds, "SQ_WAVES") / CUS, 2),
             "mean_resident_waves_per_cu": round(4 * mean(ds, "SQ_WAVE_CYCLES") / (cyc * CUS), 2),
             "max_waves_per_cu": 32,
             "valu_busy": round(4 * mean(ds, "SQ_ACTIVE_INST_VALU") / (cyc * CUS * 4), 4),
             "valu_insts": round(mean(ds, "SQ_INSTS_VALU")), "salu_insts": round(mean(ds, "SQ_INSTS_SALU")),
             "lds_insts": round(mean(ds, "SQ_INSTS_LDS"))}
        if k in f64:
            fd = f64[k]
            ops = 64 * (mean(fd, "SQ_INSTS_VALU_ADD_F64") + mean(fd, "SQ_INSTS_VALU_MUL_F64") +
                        2 * mean(fd, "SQ_INSTS_VALU_FMA_F64") + mean(fd, "SQ_INSTS_VALU_TRANS_F64"))
            e["fp64_flop_per_dispatch"] = round(ops)
            e["fp64_peak_tflops"] = FP64_PEAK_TFLOPS
        res["gn"][k] = e
    # stereo-VO kernels: tools/bench_svo.py runs a 10-pair warm-up batch and
    # then the measured 100-pair batch; the figures are the 100-pair
    # dispatch's (each kernel's last), never a mean over the two sizes
    def big(ds):
        return ds[max(ds)] if ds else None

    for k in sorted(set(sf) | set(sw)):
        if not k.startswith("svo_"):
            continue
        f, wr = big(sf.get(k, {})), big(sw.get(k, {}))
        fb = f.get("FETCH_SIZE") if f else None
        wb = wr.get("WRITE_SIZE") if wr else None
        res["svo"][k] = {"batch": "100 pairs (the last dispatch of tools/bench_svo.py)",
                         "fetch_raw_kb": round(fb, 1) if fb is not None else None,
                         "fetch_bytes": round(2 * 1024 * fb) if fb is not None else None,
                         "write_bytes": round(1024 * wb) if wb is not None else None,
                         "traffic_bytes": round(2 * 1024 * fb + 1024 * wb) if fb is not None and wb is not None else None,
                         "pmc_duration_us": round((f or wr)["_dur_ns"] / 1e3, 2)}
        q = big(sq.get(k, {}))
        if q:
            dur = q["_dur_ns"]
            cyc = dur * CLK_GHZ
            res["svo"][k].update({
                "sq_duration_us": round(dur / 1e3, 2),
                "valu_insts": round(q.get("SQ_INSTS_VALU", 0)), "salu_insts": round(q.get("SQ_INSTS_SALU", 0)),
                "lds_insts": round(q.get("SQ_INSTS_LDS", 0)),
                "valu_insts_per_us": round(q.get("SQ_INSTS_VALU", 0) / (dur / 1e3), 1),
                # SQ_ACTIVE_INST_VALU counts quad-cycles: the fraction of SIMD cycles issuing VALU
                "valu_busy": round(4 * q.get("SQ_ACTIVE_INST_VALU", 0) / (cyc * CUS * 4), 4),
                "mean_resident_waves_per_cu": round(4 * q.get("SQ_WAVE_CYCLES", 0) / (cyc * CUS), 2)})
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
