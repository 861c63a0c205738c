"""Static ISA check of the warp-specialised conv (conv3d_v5.hip): its MFMA waves
load weight fragments with inline-asm global_load_dwordx4 that the compiler's
wait insertion does not see, so no instruction may touch a destination
register before a counted s_waitcnt vmcnt has retired the load
(tools/check_asm_loads.py).  A runtime branch between such a load and its wait
let the register allocator copy the registers early (a timing-dependent wrong
result the r04 plan tests caught); this compiles the unit for gfx950 and scans
every instance.  CPU only (hipcc cross-compiles)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fast-cwdm_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_v5_async_weight_loads_have_no_early_uses(tmp_path):
    out = tmp_path / "v5.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-x", "hip", "-S", "--cuda-device-only",
                    os.path.join(CSRC, "conv3d_v5.hip"), "-o", str(out)], check=True, capture_output=True)
    text = out.read_text()
    syms = sorted({l.split(":")[0] for l in text.split("\n")
                   if l.startswith(("_ZN4cwdm16conv3d_v5_kernel", "_ZN4cwdm17conv3d_v5s_kernel"))
                   and l.split()[0].endswith(":")})
    assert len(syms) == 12, syms
    for sym in syms:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_asm_loads.py"), str(out), sym],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-2000:]
