"""Compiler-bug lint over the HIP sources (no GPU): ROCm 7.2's AMDGPU backend drops an
`and 0xffffff` (any mask of 17-24 bits) that feeds a 64-bit multiply by a non-power-of-two
constant and then multiplies the unmasked word (tools/probe/probe_mul24.hip).  Every kernel
source is compiled to LLVM IR and scanned for `mul i64 (zext (and x, M)), C` with such M, C;
decoder.hip extracts list-entry rows through an opaque v_and for this reason."""
import glob
import os
import re
import shutil
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "rnnt-inference_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def masked_wide_multiplies(ir):
    hits = []
    for fn in ir.split("\ndefine ")[1:]:  # SSA names are per function
        hits += _scan_function(fn)
    return hits


def _scan_function(ir):
    defs = {m.group(1): (m.group(2), m.group(4)) for m in
            re.finditer(r"(%[\w.]+) = (\w+)((?: nuw| nsw| nneg| disjoint)*) (?:i32|i64) ([^\n]*)", ir)}
    hits = []
    for m in re.finditer(r"(%[\w.]+) = mul(?: nuw| nsw)* i64 (%[\w.]+), (\d+)", ir):
        c = int(m.group(3))
        if c & (c - 1) == 0:
            continue
        d = defs.get(m.group(2))
        inner = re.match(r"(%[\w.]+) to", d[1]) if d and d[0] == "zext" else None
        di = defs.get(inner.group(1)) if inner else None
        mk = re.search(r", (\d+)$", di[1]) if di and di[0] == "and" else None
        if mk and (1 << 16) < int(mk.group(1)) < (1 << 24):
            hits.append(m.group(0))
    return hits


def _ir(src, out):
    flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "--cuda-device-only", "-S", "-emit-llvm"]
    if os.path.basename(src) == "encoder.hip":
        flags.append("-fno-slp-vectorize")
    subprocess.run([HIPCC, *flags, src, "-o", out], check=True, cwd=CSRC, capture_output=True)
    return open(out).read()


def test_lint_finds_the_reproducer():
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    with tempfile.TemporaryDirectory() as d:
        ir = _ir(os.path.join(REPO, "tools", "probe", "probe_mul24.hip"), os.path.join(d, "p.ll"))
    assert len(masked_wide_multiplies(ir)) >= 1


def test_no_masked_wide_multiply_in_kernels():
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    assert srcs
    with tempfile.TemporaryDirectory() as d, ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        irs = list(ex.map(lambda s: (s, _ir(s, os.path.join(d, os.path.basename(s) + ".ll"))), srcs))
    bad = {os.path.basename(s): masked_wide_multiplies(ir) for s, ir in irs}
    bad = {k: v for k, v in bad.items() if v}
    assert not bad, f"masked 24-bit values in 64-bit multiplies (miscompiled by ROCm 7.2): {bad}"
