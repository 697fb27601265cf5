"""Static check of the quick render kernels' register fence.

k_render_fwd_quick_v / _d keep the pixel's 192 channel sums in v64..v255
(v63 = the junk channel) and are compiled with amdgpu_num_vgpr(63), so the
compiler's own code must stay in v0..v62; only the kernels' inline asm may
touch v63 and above (csrc/render.hip: the index-mode zeroing, update and read,
and the two epilogues).  The attribute is a limit the compiler can overrun
without a diagnostic when register pressure rises (a hoisted-load variant
allocated v58..v72 and overwrote channels 0..8), so this disassembles the
gfx950 code object inside liblsr.so and rejects any other instruction that
names a register at or above v63.

    python tools/check_vgpr_fence.py [liblsr.so]     (exit 1 on a violation)
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin/llvm-objdump"
HI = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")

# the inline-asm forms allowed to name v63 and above (render.hip); each form also
# pins which operands may be high: addresses and offsets below v63, data only in
# the channel registers v64..v255 (a compiler-made store with a spilled address
# or data in the fence, the overrun this tool exists to catch, is rejected)
ALLOWED = [
    re.compile(r"^v_fma_f32 v63, v(\d+), v(\d+), v63$"),                 # LSR_QV_WORD (index mode)
    re.compile(r"^v_mov_b32(_e32)? v63, 0$"),                             # accumulator zeroing (index mode)
    re.compile(r"^v_mov_b32(_e32)? v(\d+), v64$"),                        # index-mode read (epilogue loop)
    re.compile(r"^global_store_dwordx4 v\[(\d+):(\d+)\], v\[(\d+):(\d+)\], off( offset:\d+)?$"),   # LSR_QHWC
    re.compile(r"^buffer_store_dword v(\d+), v(\d+), s\[\d+:\d+\], s\d+ offen$"),                   # LSR_QEPI
]


def _regs(text):
    out = []
    for m in HI.finditer(text):
        if m.group(1):
            out.append(int(m.group(1)))
        else:
            out.extend(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def _allowed(ins):
    for k, p in enumerate(ALLOWED):
        m = p.match(ins)
        if not m:
            continue
        if k == 0:
            return int(m.group(1)) < 63 and int(m.group(2)) < 63
        if k == 1:
            return True
        if k == 2:
            return int(m.group(2)) < 63
        if k == 3:   # address pair below v63, data a 4-aligned quad inside v64..v255
            a0, a1, d0, d1 = (int(m.group(i)) for i in range(1, 5))
            return a1 == a0 + 1 and a1 < 63 and d0 >= 64 and d0 % 4 == 0 and d1 == d0 + 3 and d1 <= 255
        if k == 4:   # data one channel register, offset register below v63
            return 64 <= int(m.group(1)) <= 255 and int(m.group(2)) < 63
    return False


def check(lib=None):
    """[(kernel, instruction)] of every instruction of a quick render kernel
    that names v63+ outside the allowed asm forms; raises if nothing was
    checked (no quick kernel found)."""
    lib = lib or os.path.join(ROOT, "langsplatv2_amd", "liblsr.so")
    bad, seen = [], 0
    with tempfile.TemporaryDirectory() as d:
        dst = os.path.join(d, "lib.so")
        with open(lib, "rb") as f, open(dst, "wb") as g:
            g.write(f.read())
        subprocess.run([LLVM, "--offloading", dst], cwd=d, check=True, capture_output=True)
        for co in sorted(glob.glob(os.path.join(d, "lib.so.*gfx950*"))):
            if os.path.getsize(co) == 0:
                continue
            txt = subprocess.run([LLVM, "-d", "--mcpu=gfx950", "--no-show-raw-insn", co], check=True,
                                 capture_output=True, text=True).stdout
            kern = None
            for line in txt.splitlines():
                if line.endswith(">:"):
                    name = line.split("<", 1)[1][:-2]
                    kern = name if "k_render_fwd_quick" in name else None
                    if kern:
                        seen += 1
                    continue
                if kern is None:
                    continue
                ins = line.strip().split("//")[0].strip()
                if not ins or ins.startswith(";"):
                    continue
                if any(r >= 63 for r in _regs(ins)) and not _allowed(ins):
                    bad.append((kern, ins))
    if seen == 0:
        raise RuntimeError("no quick render kernel found in the code objects")
    return bad


if __name__ == "__main__":
    v = check(sys.argv[1] if len(sys.argv) > 1 else None)
    for k, i in v[:40]:
        print(f"{k}: {i}")
    print(f"{len(v)} violation(s)")
    sys.exit(1 if v else 0)
