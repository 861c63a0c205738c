"""Static ISA check of the warp-specialised conv (conv3d_v5.hip): its MFMA waves
load weight fragments with inline-asm global_load_dwordx4 that the compiler's
wait insertion does not see, so no instruction may touch a destination
register before a counted s_waitcnt vmcnt has retired the load
(tools/check_asm_loads.py).  A runtime branch between such a load and its wait
let the register allocator copy the registers early (a timing-dependent wrong
result the r04 plan tests caught); this compiles the unit for gfx950 and scans
every instance, following branches and loop back-edges to a fixpoint (a load
issued at a loop's tail is in flight at its head on the next trip).  The
checker itself is pinned by hazardous / clean snippets.  CPU only (hipcc
cross-compiles)."""
import os
import shutil
import subprocess
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import check_asm_loads as cal  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fast-cwdm_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_v5_async_weight_loads_have_no_early_uses(tmp_path):
    out = tmp_path / "v5.s"
    # the Makefile's flags for this unit
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-fno-slp-vectorize", "-munsafe-fp-atomics",
                    "-x", "hip", "-S", "--cuda-device-only",
                    os.path.join(CSRC, "conv3d_v5.hip"), "-o", str(out)], check=True, capture_output=True)
    text = out.read_text()
    syms = sorted({l.split(":")[0] for l in text.split("\n")
                   if l.startswith(("_ZN4cwdm16conv3d_v5_kernel", "_ZN4cwdm17conv3d_v5s_kernel"))
                   and l.split()[0].endswith(":")})
    assert len(syms) == 16, syms
    for sym in syms:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_asm_loads.py"), str(out), sym],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-2000:]


def _lines(src):
    return list(enumerate(src.strip("\n").split("\n"), 1))


# a weight load issued at the loop's tail and read at its head on the next trip:
# the entry path waits, the back-edge does not -- invisible to a linear scan
_LOOP_HAZARD = """
\tglobal_load_dwordx4 v[0:3], v[10:11], off
\ts_waitcnt vmcnt(0)
.LBB0_1:
\tv_mov_b32 v20, v0
\tv_add_u32 v30, v30, v31
\tglobal_load_dwordx4 v[0:3], v[10:11], off
\ts_cbranch_scc1 .LBB0_1
\ts_waitcnt vmcnt(0)
\ts_endpgm
"""


def test_checker_flags_a_loop_carried_hazard():
    assert cal.check(_lines(_LOOP_HAZARD), verbose=False) == 1


def test_checker_accepts_the_waited_loop():
    ok = _LOOP_HAZARD.replace(".LBB0_1:\n", ".LBB0_1:\n\ts_waitcnt vmcnt(0)\n")
    assert cal.check(_lines(ok), verbose=False) == 0
    # a counted wait that leaves only a younger, untouched load in flight is fine too
    counted = _LOOP_HAZARD.replace("\tglobal_load_dwordx4 v[0:3], v[10:11], off\n\ts_cbranch",
                                   "\tglobal_load_dwordx4 v[0:3], v[10:11], off\n"
                                   "\tglobal_load_dwordx4 v[4:7], v[10:11], off\n\ts_waitcnt vmcnt(1)\n\ts_cbranch")
    assert cal.check(_lines(counted), verbose=False) == 0


def test_checker_flags_a_hazard_on_one_branch_only():
    src = """
\tglobal_load_dwordx4 v[0:3], v[10:11], off
\ts_cbranch_scc0 .LBB0_2
\ts_waitcnt vmcnt(0)
.LBB0_2:
\tv_mov_b32 v20, v2
\ts_endpgm
"""
    assert cal.check(_lines(src), verbose=False) == 1
    assert cal.check(_lines(src.replace("\ts_cbranch_scc0 .LBB0_2\n", "")), verbose=False) == 0
