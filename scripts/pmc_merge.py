#!/usr/bin/env python3
"""Merge rocprofv3 --pmc pass summaries (pmc_summary.py outputs) into the per-kernel file
bench.py reads (profiles/pmc_<config>.json).
usage: pmc_merge.py <config> <fetch.json> <write.json> <out.json> [sq_pass.json ...]

HBM: read = 2*1024*FETCH_SIZE (gfx950 half-count correction for 16-byte streaming loads,
MI355X_MICROARCH.md HBM), write = 1024*WRITE_SIZE, per dispatch.
SQ passes (each with GRBM_GUI_ACTIVE, so every ratio below uses the cycles of its own pass):
  cycles          GRBM_GUI_ACTIVE / 8 (sum over the 8 XCDs)
  valu_issue_util 2 * SQ_INSTS_VALU / (1024 SIMDs * cycles): a wave64 VALU op holds a SIMD-32
                  for 2 cycles (MI355X_MICROARCH.md "Wave scheduling"); multi-pass 64-bit ops
                  (v_mad_u64_u32, 64-bit shifts) make this a lower bound
  valu_cycle_util_est  the same with SQ_INSTS_VALU_INT64 instructions at 8 cycles (v_mad_u64_u32
                  is quarter rate: tests/microbench/mac_rate.hip) -- an upper estimate
  lds_util        SQ_LDS_IDX_ACTIVE / (256 CUs * cycles)
  wait_*_frac     SQ_WAIT_INST_ANY, SQ_WAIT_ANY over SQ_WAVE_CYCLES (quad-cycles both)
  waves_per_simd  4 * SQ_WAVE_CYCLES / (1024 * cycles): mean resident waves per SIMD
  clock_ghz       cycles / the pass's own kernel duration, when the summary carries one"""
import json
import sys

cfg, fj, wj, out = sys.argv[1:5]
sq = [json.load(open(p)) for p in sys.argv[5:]]
f, w = json.load(open(fj)), json.load(open(wj))
kern = {}
for k in sorted(set(f) | set(w) | set().union(*[set(s) for s in sq])):
    rd = f.get(k, {}).get("hbm_read_bytes_corrected")
    wr = w.get(k, {}).get("hbm_write_bytes")
    rec = {"dispatches": f.get(k, w.get(k, {})).get("dispatches")}
    if rd is not None:
        rec["hbm_read_bytes_per_launch"] = rd
    if wr is not None:
        rec["hbm_write_bytes_per_launch"] = wr
    if rd is not None and wr is not None:
        rec["hbm_bytes_per_launch"] = rd + wr
    for s in sq:
        r = s.get(k)
        if not r or not r.get("GRBM_GUI_ACTIVE"):
            continue
        cyc = r["GRBM_GUI_ACTIVE"] / 8
        for c, v in r.items():
            if c.startswith("SQ_"):
                rec[c] = v
        if "SQ_INSTS_VALU" in r:
            rec["valu_issue_util"] = 2 * r["SQ_INSTS_VALU"] / (1024 * cyc)
            if "SQ_INSTS_VALU_INT64" in r:   # 64-bit integer ops (v_mad_u64_u32 ...) priced at 8 cycles
                i64 = r["SQ_INSTS_VALU_INT64"]
                rec["valu_cycle_util_est"] = (2 * (r["SQ_INSTS_VALU"] - i64) + 8 * i64) / (1024 * cyc)
        if "SQ_LDS_IDX_ACTIVE" in r:
            rec["lds_util"] = r["SQ_LDS_IDX_ACTIVE"] / (256 * cyc)
        if "SQ_WAVE_CYCLES" in r:
            rec["waves_per_simd"] = 4 * r["SQ_WAVE_CYCLES"] / (1024 * cyc)
            for c, n in (("SQ_WAIT_INST_ANY", "wait_inst_frac"), ("SQ_WAIT_ANY", "wait_any_frac")):
                if c in r:
                    rec[n] = r[c] / r["SQ_WAVE_CYCLES"]
        if r.get("duration_ns"):
            rec["clock_ghz"] = cyc / r["duration_ns"]
    kern[k] = rec
json.dump({"config": cfg,
           "method": "rocprofv3 --pmc passes over `bench.py --config "
                     f"{cfg} --steps 1 --warmup 0` (FETCH_SIZE, WRITE_SIZE and each SQ set in a pass of its own); "
                     "per dispatch averages; derived fields: scripts/pmc_merge.py docstring",
           "source": ", ".join(sys.argv[2:4] + sys.argv[5:]), "kernels": kern}, open(out, "w"), indent=1)
