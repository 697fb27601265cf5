"""The quick render register-fence checker (tools/check_vgpr_fence.py, run by
__graft_entry__.build()) accepts only the inline-asm forms render.hip emits:
synthetic disassembly lines a compiler-made overrun would produce are rejected
(the store forms used to be accepted whatever their operands)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import check_vgpr_fence as F  # noqa: E402


@pytest.mark.parametrize("ins", [
    "v_fma_f32 v63, v12, v40, v63",
    "v_mov_b32_e32 v63, 0",
    "v_mov_b32_e32 v5, v64",
    "global_store_dwordx4 v[2:3], v[64:67], off",
    "global_store_dwordx4 v[60:61], v[252:255], off offset:752",
    "buffer_store_dword v64, v7, s[8:11], s2 offen",
    "buffer_store_dword v255, v62, s[8:11], s2 offen",
])
def test_emitted_forms_pass(ins):
    assert F._allowed(ins)


@pytest.mark.parametrize("ins", [
    "v_fma_f32 v63, v70, v40, v63",                          # a channel register as an operand
    "global_store_dwordx4 v[64:65], v[68:71], off",          # address in the fence
    "global_store_dwordx4 v[2:3], v[62:65], off",            # data straddling v63
    "global_store_dwordx4 v[2:3], v[66:69], off",            # data quad not 4-aligned
    "global_store_dwordx4 v[2:4], v[64:67], off",            # not an address pair
    "buffer_store_dword v70, v63, s[8:11], s2 offen",        # offset register in the fence
    "buffer_store_dword v40, v7, s[8:11], s2 offen",         # data outside the channel registers
    "v_add_f32_e32 v70, v1, v2",                             # any other instruction naming v63+
    "global_load_dwordx4 v[64:67], v[2:3], off",
])
def test_overruns_rejected(ins):
    assert not F._allowed(ins)
