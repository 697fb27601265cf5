"""The quick render kernels keep each pixel's 192 channel sums in v64..v255
and limit the compiler to v0..v62 (amdgpu_num_vgpr(63), csrc/render.hip); the
compiler can overrun that limit silently under register pressure.  The built
library's gfx950 code object is disassembled and every instruction outside the
kernels' inline asm must stay below v63 (tools/check_vgpr_fence.py)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_vgpr_fence  # noqa: E402


@pytest.mark.skipif(not os.path.exists(check_vgpr_fence.LLVM), reason="llvm-objdump not installed")
def test_quick_kernels_respect_the_register_fence():
    assert check_vgpr_fence.check() == []


@pytest.mark.skipif(not os.path.exists(check_vgpr_fence.LLVM), reason="llvm-objdump not installed")
def test_fence_rules():
    ok = check_vgpr_fence._allowed
    assert ok("v_fma_f32 v63, v44, v12, v63")
    assert not ok("v_fma_f32 v63, v64, v12, v63")          # a compiler value in an accumulator register
    assert ok("buffer_store_dword v200, v0, s[0:3], s5 offen")
    assert ok("global_store_dwordx4 v[2:3], v[64:67], off offset:16")
    assert not ok("v_readfirstlane_b32 s69, v72")
