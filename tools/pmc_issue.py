"""Issue-rate roofline of the render kernels from two rocprofv3 SQ passes
(tools/pass.py pmc: P1 = instruction counts + SQ_BUSY_CYCLES + SQ_WAVE_CYCLES,
P2 = wait / active / MFMA-busy cycles), per kernel, averaged per dispatch.

Units (MI355X_MICROARCH.md, rocprofv3 PMC + cycle-constants rows):
  * SQ_BUSY_CYCLES is summed over the 32 shader engines -> kernel cycles =
    SQ_BUSY_CYCLES / 32; SIMD-cycles = kernel cycles x 1024 SIMDs;
  * SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles, summed
    over waves; SQ_VALU_MFMA_BUSY_CYCLES counts cycles, summed over SIMDs;
  * a wave64 VALU instruction occupies a SIMD-32 for 2 cycles at full rate
    (one wave alone issues one per 4), so the VALU pipe's issue utilisation
    is SQ_INSTS_VALU x 2 / SIMD-cycles.

Derived (per kernel): valu_issue_frac (VALU pipe busy, the rate roofline),
valu_active_frac (SQ_ACTIVE_INST_VALU x 4 / SIMD-cycles: summed per-wave
issue occupancy), mfma_busy_frac, waves_per_simd (average resident), and the
split of wave-cycles into issuing / issue-stalled (dependency, arbitration) /
parked in s_waitcnt.

Usage: python tools/pmc_issue.py P1_DIR P2_DIR OUT.json [--units KERNEL=N ...]
  --units: per-dispatch work units of a kernel (e.g. staged (candidate,
  8x8-block) pairs) -> instructions per unit."""
import csv
import json
import re
import sys
from collections import defaultdict

SIMDS = 1024
SES = 32


def short(name: str) -> str:
    n = name.replace("void ", "").split("(")[0]
    return re.sub(r"^lsr::", "", n)


def per_kernel(path: str) -> dict:
    acc = defaultdict(lambda: defaultdict(float))
    names = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            d = int(row["Dispatch_Id"])
            acc[d][row["Counter_Name"]] += float(row["Counter_Value"])
            names[d] = short(row["Kernel_Name"])
    out = defaultdict(lambda: {"n": 0, "c": defaultdict(float)})
    for d, cs in acc.items():
        k = out[names[d]]
        k["n"] += 1
        for c, v in cs.items():
            k["c"][c] += v
    return {k: {"dispatches": v["n"], "counters": {c: x / v["n"] for c, x in v["c"].items()}} for k, v in out.items()}


def derive(c: dict) -> dict:
    busy = c.get("SQ_BUSY_CYCLES", 0.0) / SES
    simd = busy * SIMDS
    if simd <= 0:
        return {}
    d = {"kernel_cycles": round(busy), "simd_cycles": round(simd)}
    if "SQ_INSTS_VALU" in c:
        d["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] * 2 / simd, 4)
    if "SQ_ACTIVE_INST_VALU" in c:
        d["valu_active_frac"] = round(c["SQ_ACTIVE_INST_VALU"] * 4 / simd, 4)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        d["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd, 4)
    if "SQ_INSTS_SALU" in c:
        d["salu_issue_frac"] = round(c["SQ_INSTS_SALU"] / simd, 4)
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    if wc > 0:
        d["waves_per_simd"] = round(wc * 4 / simd, 3)
        for k, nm in (("SQ_ACTIVE_INST_ANY", "wave_issuing"), ("SQ_WAIT_INST_ANY", "wave_issue_stalled"),
                      ("SQ_WAIT_ANY", "wave_in_waitcnt")):
            if k in c:
                d[nm + "_frac"] = round(c[k] / wc, 4)
    return d


def main():
    args = sys.argv[1:]
    units = {}
    if "--units" in args:
        i = args.index("--units")
        for a in args[i + 1:]:
            k, v = a.split("=", 1)
            units[k] = float(v)
        args = args[:i]
    p1, p2, out = args[:3]
    a = per_kernel(f"{p1}/run_counter_collection.csv")
    b = per_kernel(f"{p2}/run_counter_collection.csv")
    res = {}
    for k in sorted(set(a) & set(b)):
        c = dict(a[k]["counters"])
        c.update(b[k]["counters"])
        d = derive(c)
        for uk, u in units.items():
            if k.startswith(uk) and u > 0:
                d["units_per_dispatch"] = u
                for ck, nm in (("SQ_INSTS_VALU", "valu_per_unit"), ("SQ_INSTS_MFMA", "mfma_per_unit"),
                               ("SQ_INSTS_SALU", "salu_per_unit"), ("SQ_INSTS_LDS", "lds_per_unit")):
                    if ck in c:
                        d[nm] = round(c[ck] / u, 2)
        res[k] = {"dispatches": min(a[k]["dispatches"], b[k]["dispatches"]),
                  "counters": {ck: round(v) for ck, v in sorted(c.items())}, "derived": d}
    doc = {"method": "rocprofv3 --pmc, two SQ passes (tools/pass.py pmc) over tools/pmc_step.py; per-dispatch averages; "
                     "see tools/pmc_issue.py for the units", "kernels": res}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for k, v in res.items():
        if k.startswith("k_render") or k.startswith("k_quick"):
            print(k, json.dumps(v["derived"]))


if __name__ == "__main__":
    main()
