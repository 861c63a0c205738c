"""CPU oracle for the fast-cwdm hot path -- TEST INFRASTRUCTURE ONLY.

This package is a PyTorch-CPU fp32 (float64 for the schedule tables)
restatement of the reference's DWT -> U-Net -> IDWT diffusion path, written
against the reference files cited in each function's docstring
(/root/reference is read as text only; importing it is denied).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker.  The
product path (``fast-cwdm_amd/``) never imports it and has no CPU fallback.

Pinning: the Haar filter bank is pinned against PyWavelets 1.1.1 (the
library the reference takes its taps from, ``DWT_IDWT/DWT_IDWT_layer.py:451-457``)
through ``tests/golden/pywt_haar3d.npz`` (script ``oracle/gen_pywt_golden.py``),
and by the analytic known-answer tests of SURVEY.md §4.  The diffusion tables
are pinned by closed-form float64 recomputation.  The U-Net and the sampler
loop have no reference fixture (the reference ships none and cannot be run
here): for those the oracle is a line-by-line restatement, "parity unpinned"
against the reference itself, and the committed fixtures in ``tests/golden``
freeze its outputs.
"""
