"""One GPU-box measurement pass (repo root, under gpurun): the recipes the
round-specific shell scripts of rounds 1-5 repeated, as named steps.

    python tools/pass.py TAG STEP [STEP ...]

Steps (run in order; outputs under gpurun_out/, named TAG_*):
    tests          pytest -m gpu (all); failures are reported and the pass goes on
    ftests         pytest tests/test_fullsize.py (whole BASELINE frames)
    test:PATH      pytest PATH (one file or node id)
    smoke          __graft_entry__.smoke()
    bench          python bench.py                       -> TAG_bench.json
    cfg1 cfg2 cfg5 python bench.py --config N            -> TAG_cfgN.json
    prof           rocprofv3 --kernel-trace --stats of the cfg3 step ALONE
                   (bench.py --no-quick --no-fwd-1mpix --no-det --no-cpu-baseline)
                   -> TAG_kernel_stats.md (the roofline cross-check)
    profq          the same over the quick path only (tools/pmc_step.py LSR_QUICK=1)
    pmc            cfg3: two SQ issue passes + FETCH_SIZE / WRITE_SIZE passes over
                   tools/pmc_step.py -> TAG_pmc_issue.json, TAG_pmc_traffic.json
    pmcdet         pmc's four passes with the deterministic backward -> det_TAG_pmc_*.json
                   (named apart from the r* files bench.py reads)
    pmc2 pmc5      FETCH / WRITE passes at cfg2 / cfg5 -> cfgN_TAG_pmc_traffic.json
    rehearse2      bench.py --gpus 2 on the one-GPU box (gloo exchange, both ranks on cuda:0)
    ab:NAME=LIB,.. tools/ab.py A/B of library variants (tools/variant.py builds them)
                   in one process, both orders; LSR_CFG picks the config

Every step runs under its own time limit.  A step whose checks fail (exit 1)
does not stop the pass; a crash, abort, signal or time limit ends it there, so
nothing more touches the GPU after a fault.  Each rocprofv3 counter pass is
its own run (rocprofv3 does not split counters over passes), with the program
right after `--`."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PY = sys.executable
SQ1 = "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH"
SQ2 = ("SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES "
       "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR")
CFG3_ONLY = ["--steps", "20", "--warmup", "5", "--no-cpu-baseline", "--no-fwd-1mpix", "--no-quick", "--no-det"]


class Fault(Exception):
    pass


def run(cmd, limit, log, env=None, cwd=ROOT, kill=False):
    """cmd (argv) under `timeout`; stdout+stderr to log.  Returns its status;
    raises Fault on anything but 0 / 1."""
    tl = ["timeout", "-s", "KILL", str(limit)] if kill else ["timeout", "-k", "10", str(limit)]
    e = dict(os.environ)
    e.setdefault("TMPDIR", "/tmp")
    e.update(env or {})
    print(f"[pass] {' '.join(cmd)}  > {os.path.relpath(log, ROOT)}", flush=True)
    with open(log, "w") as f:
        rc = subprocess.call(tl + cmd, stdout=f, stderr=subprocess.STDOUT, env=e, cwd=cwd)
    print(f"[pass] rc={rc}", flush=True)
    if rc not in (0, 1):
        with open(log) as f:
            print("".join(f.readlines()[-30:]))
        raise Fault(f"{cmd[0]} ended with status {rc}")
    return rc


def tail(path, n=8):
    with open(path) as f:
        print("".join(l for l in f.readlines()[-n:] if "amdgpu.ids" not in l), flush=True)


def pytest(tag, name, target, limit=1000):
    log = os.path.join(OUT, f"{tag}_{name}.log")
    run([PY, "-u", "-m", "pytest", target, "-m", "gpu", "-v", "--timeout", "400", "--timeout-method", "thread",
         "--durations=15"], limit, log)
    tail(log, 20)


def bench(tag, name, args, limit=600):
    js = os.path.join(OUT, f"{tag}_{name}.json")
    err = js[:-5] + ".err"
    tl = ["timeout", "-k", "10", str(limit)]
    with open(js, "w") as f, open(err, "w") as g:
        rc = subprocess.call(tl + [PY, "bench.py"] + args, stdout=f, stderr=g, cwd=ROOT)
    if rc != 0:
        tail(err, 20)
        raise Fault(f"bench {name} ended with status {rc}")
    tail(js, 1)


def rocprof(tag, name, counters, prog, limit=180, env=None):
    d = os.path.join(OUT, f"{tag}_{name}")
    args = ["rocprofv3"] + (["--pmc"] + counters.split() if counters else ["--kernel-trace", "--stats"])
    args += ["-d", d, "-o", "run"] + (["--output-format", "csv"] if counters else []) + ["--"] + prog
    run(args, limit, d + ".log", env=env, cwd="/tmp", kill=bool(counters))
    return d


def step(tag, s):
    os.makedirs(OUT, exist_ok=True)
    if s == "tests":
        pytest(tag, "tests", "tests")
    elif s == "ftests":
        pytest(tag, "ftests", "tests/test_fullsize.py")
    elif s.startswith("test:"):
        pytest(tag, "t_" + os.path.basename(s[5:]).split(".")[0].split(":")[0], s[5:], limit=600)
    elif s == "smoke":
        log = os.path.join(OUT, f"{tag}_smoke.log")
        run([PY, "-u", "-c", "import __graft_entry__ as g; g.smoke()"], 300, log)
        tail(log, 3)
    elif s == "bench":
        bench(tag, "bench", [])
    elif s in ("cfg1", "cfg2", "cfg5"):
        bench(tag, s, ["--config", s[3:]])
    elif s == "prof":
        d = rocprof(tag, "prof", None, ["python3", os.path.join(ROOT, "bench.py")] + CFG3_ONLY, limit=300)
        db = next((os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f == "run_results.db"), None)
        md = os.path.join(OUT, f"{tag}_kernel_stats.md")
        subprocess.call([PY, "tools/prof_summary.py", db or "", md,
                         f"{tag}: bench.py {' '.join(CFG3_ONLY)} (cfg3 step alone) under rocprofv3 --kernel-trace --stats"],
                        cwd=ROOT, stdout=subprocess.DEVNULL)
        tail(md, 14)
    elif s == "profq":
        d = rocprof(tag, "profq", None, ["python3", os.path.join(ROOT, "tools", "pmc_step.py")], limit=300,
                    env={"LSR_QUICK": "1", "LSR_STEPS": "20"})
        db = next((os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f == "run_results.db"), None)
        md = os.path.join(OUT, f"{tag}_quick_kernel_stats.md")
        subprocess.call([PY, "tools/prof_summary.py", db or "", md,
                         f"{tag}: quick path alone (tools/pmc_step.py LSR_QUICK=1) under rocprofv3 --kernel-trace --stats"],
                        cwd=ROOT, stdout=subprocess.DEVNULL)
        tail(md, 10)
    elif s == "pmc":
        prog = ["python3", os.path.join(ROOT, "tools", "pmc_step.py")]
        env = {"LSR_STEPS": "2"}
        s1 = rocprof(tag, "sq1", SQ1, prog, env=env)
        s2 = rocprof(tag, "sq2", SQ2, prog, env=env)
        fF = rocprof(tag, "pmcF", "FETCH_SIZE", prog, env=env)
        fW = rocprof(tag, "pmcW", "WRITE_SIZE", prog, env=env)
        units = subprocess.run([PY, "tools/lst_units.py"], cwd=ROOT, capture_output=True, text=True).stdout.strip()
        units = units or "3490000"
        with open(os.path.join(OUT, f"{tag}_pmc_issue.txt"), "w") as f:
            subprocess.call([PY, "tools/pmc_issue.py", s1, s2, os.path.join(OUT, f"{tag}_pmc_issue.json"),
                             "--units", f"k_render_bwd_mf={units}"], cwd=ROOT, stdout=f)
        with open(os.path.join(OUT, f"{tag}_pmc_traffic.txt"), "w") as f:
            subprocess.call([PY, "tools/pmc_traffic.py", fF, fW, os.path.join(OUT, f"{tag}_pmc_traffic.json")],
                            cwd=ROOT, stdout=f)
        tail(os.path.join(OUT, f"{tag}_pmc_issue.txt"), 6)
        tail(os.path.join(OUT, f"{tag}_pmc_traffic.txt"), 12)
    elif s == "pmcdet":
        prog = ["python3", os.path.join(ROOT, "tools", "pmc_step.py")]
        env = {"LSR_STEPS": "2", "LSR_DET": "1"}
        s1 = rocprof(tag, "dsq1", SQ1, prog, env=env)
        s2 = rocprof(tag, "dsq2", SQ2, prog, env=env)
        fF = rocprof(tag, "dpmcF", "FETCH_SIZE", prog, env=env)
        fW = rocprof(tag, "dpmcW", "WRITE_SIZE", prog, env=env)
        with open(os.path.join(OUT, f"det_{tag}_pmc_issue.txt"), "w") as f:
            subprocess.call([PY, "tools/pmc_issue.py", s1, s2, os.path.join(OUT, f"det_{tag}_pmc_issue.json")],
                            cwd=ROOT, stdout=f)
        with open(os.path.join(OUT, f"det_{tag}_pmc_traffic.txt"), "w") as f:
            subprocess.call([PY, "tools/pmc_traffic.py", fF, fW, os.path.join(OUT, f"det_{tag}_pmc_traffic.json")],
                            cwd=ROOT, stdout=f)
        tail(os.path.join(OUT, f"det_{tag}_pmc_issue.txt"), 12)
        tail(os.path.join(OUT, f"det_{tag}_pmc_traffic.txt"), 12)
    elif s in ("pmc2", "pmc5"):
        n = s[3:]
        prog = ["python3", os.path.join(ROOT, "tools", "pmc_step.py")]
        env = {"LSR_STEPS": "2", "LSR_CFG": n}
        fF = rocprof(tag, f"c{n}F", "FETCH_SIZE", prog, env=env)
        fW = rocprof(tag, f"c{n}W", "WRITE_SIZE", prog, env=env)
        txt = os.path.join(OUT, f"cfg{n}_{tag}_pmc_traffic.txt")
        with open(txt, "w") as f:
            subprocess.call([PY, "tools/pmc_traffic.py", fF, fW, os.path.join(OUT, f"cfg{n}_{tag}_pmc_traffic.json")],
                            cwd=ROOT, stdout=f)
        tail(txt, 12)
    elif s == "rehearse2":
        # bench.py's multi-rank path on the one-GPU box: two ranks on cuda:0 with a gloo
        # exchange (rehearsal-only overrides; the driver's runs use RCCL, one GPU per rank)
        js = os.path.join(OUT, f"{tag}_rehearse2.json")
        env = dict(os.environ, LSR_BENCH_BACKEND="gloo", LSR_BENCH_SAME_DEVICE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
        with open(js, "w") as f, open(js[:-5] + ".err", "w") as g:
            rc = subprocess.call(["timeout", "-k", "10", "400", PY, "bench.py", "--gpus", "2", "--steps", "5",
                                  "--warmup", "2", "--no-quick", "--no-fwd-1mpix", "--no-cpu-baseline", "--no-det"],
                                 stdout=f, stderr=g, cwd=ROOT, env=env)
        if rc != 0:
            tail(js[:-5] + ".err", 20)
            raise Fault(f"rehearse2 ended with status {rc}")
        tail(js, 1)
    elif s.startswith("ab:"):
        pairs = s[3:].split(",")
        name = "_".join(p.split("=")[0] for p in pairs)
        for order, ps in (("", pairs), ("_rev", pairs[::-1])):
            log = os.path.join(OUT, f"{tag}_ab_{name}{order}.txt")
            run([PY, "-u", "tools/ab.py"] + ps, 600, log)
            tail(log, len(pairs) + 2)
    else:
        raise SystemExit(f"unknown step {s}")


def main():
    if len(sys.argv) < 3:
        raise SystemExit(__doc__)
    tag = sys.argv[1]
    try:
        for s in sys.argv[2:]:
            print(f"== {s}", flush=True)
            step(tag, s)
    except Fault as e:
        print(f"[pass] stopped: {e}", flush=True)
        return 2
    print(f"pass {tag} done", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
