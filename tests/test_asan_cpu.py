"""Host-side AddressSanitizer + UBSan over the C ABI's host logic (no GPU):
the U-Net plan builder for every supported configuration family (run.sh,
resblock_updown=False, WavUNetModel incl. the reused decoder blocks, config
5's 3-level model) and the error paths of cwdm_unet_create.  The sanitized
build (tests/asan/build.sh, ~2 min on 8 cores) is cached by source hash under
fast-cwdm_amd/build/asan/ (__graft_entry__.build() prepares it)."""
import os
import subprocess
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "fast-cwdm_amd"))


def asan_binary():
    from cwdm_hip.srchash import source_hash
    out = os.path.join(ROOT, "fast-cwdm_amd", "build", "asan", source_hash())
    exe = os.path.join(out, "plan_asan")
    drv = os.path.join(ROOT, "tests", "asan", "plan_asan.cpp")
    if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(drv):
        subprocess.run(["bash", os.path.join(ROOT, "tests", "asan", "build.sh"), out], check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=900)
    return exe


def test_plan_host_logic_under_asan_ubsan():
    exe = asan_binary()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "plan_asan: ok" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
