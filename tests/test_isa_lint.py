"""Compiler-bug lint over the HIP sources (no GPU): ROCm 7.2's AMDGPU backend drops an
`and 0xffffff` (any mask of 17-24 bits) that feeds a 64-bit multiply by a non-power-of-two
constant and then multiplies the unmasked word (tools/probe/probe_mul24.hip).  Every kernel
source is compiled to LLVM IR and scanned for a `mul i64 V, C` (C not a power of two) whose
operand V derives from such an `and` through zext / sext / shl / or / add / mul -- the direct form
`mul i64 (zext (and x, M)), C` and the chain form `((size_t)(x & M) * 2 + s) * C` alike.  Round 3's
main extracted rows with a plain mask and had 16 such multiplies (the chain form); decoder.hip
now extracts every list-entry row through the opaque v_and of `entry_row`."""
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


# integer operations a masked value may pass through on its way into the wide multiply (the
# backend's 24-bit multiply matching looks through the same shifts / ors / adds / extensions:
# ((size_t)(e & M) * 2 + slot) * 1280 is `mul i64 (or (shl (zext (and e, M)), 1), slot), 1280`)
_PASS = {"zext", "sext", "shl", "or", "add", "mul", "trunc"}


def _masked_source(name, defs, depth=0):
    """The 17..24-bit `and` mask that `name` is derived from through _PASS ops, or None."""
    d = defs.get(name)
    if d is None or depth > 8:
        return None
    op, rest = d
    if op == "and":
        mk = re.search(r", (\d+)$", rest)
        if mk and (1 << 16) < int(mk.group(1)) < (1 << 24):
            return int(mk.group(1))
        return None
    if op not in _PASS:
        return None
    for operand in re.findall(r"(%[\w.]+)", rest):
        m = _masked_source(operand, defs, depth + 1)
        if m is not None:
            return m
    return None


def _scan_function(ir):
    defs = {m.group(1): (m.group(2), m.group(4)) for m in
            re.finditer(r"(%[\w.]+) = (\w+)((?: nuw| nsw| nneg| disjoint| exact)*) (?:i8|i16|i32|i64) ([^\n]*)", ir)}
    hits = []
    for m in re.finditer(r"(%[\w.]+) = mul(?: nuw| nsw)* i64 (%[\w.]+), (\d+)", ir):
        c = int(m.group(3))
        if c & (c - 1) == 0:
            continue
        if _masked_source(m.group(2), defs) is not None:
            hits.append(m.group(0))
    return hits


def test_lint_sees_through_shl_or():
    """The chain form (row * 2 + slot) * 1280 is flagged as well as the direct one."""
    ir = ("\ndefine void @f(i32 %e, i64 %s) {\n"
          "  %a = and i32 %e, 16777215\n"
          "  %z = zext nneg i32 %a to i64\n"
          "  %h = shl nuw nsw i64 %z, 1\n"
          "  %o = or disjoint i64 %h, %s\n"
          "  %m = mul nuw nsw i64 %o, 1280\n"
          "  ret void\n}\n")
    assert masked_wide_multiplies(ir) == ["%m = mul nuw nsw i64 %o, 1280"]
    assert masked_wide_multiplies(ir.replace("16777215", "65535")) == []


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


def test_featurizer_has_no_packed_fp32():
    """featurizer.hip is built with -fno-slp-vectorize (Makefile): packed FP32 VALU
    (v_pk_add / mul / fma_f32) in fz_logmel's FFT gave wrong results in lanes 48-63 of a wave while
    decode step kernels shared the CU (tools/r04_fzdiag.sh, the corrupted frames move
    with those lanes; without packed FP32 0 of ~100k batches).  The gfx950 ISA of the file, built
    with the Makefile's flags, must not contain them."""
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    mk = open(os.path.join(CSRC, "Makefile")).read()
    assert re.search(r"^featurizer\.o: FLAGS \+= -fno-slp-vectorize", mk, re.M), "Makefile lost the featurizer flag"
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "fz.s")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-w",
                        "-fno-slp-vectorize", "--cuda-device-only", "-S", "featurizer.hip", "-o", out],
                       check=True, cwd=CSRC, capture_output=True)
        isa = open(out).read()
    assert "fz_logmel_kernel" in isa
    hits = re.findall(r"^\s*(v_pk_(?:add|mul|fma)_f32)\b", isa, re.M)
    assert not hits, f"packed FP32 in featurizer.hip's ISA: {sorted(set(hits))}"
