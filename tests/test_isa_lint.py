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
    if os.path.dirname(os.path.abspath(src)) == CSRC:
        flags += _nopk_flags()
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


PACKED_FP32 = re.compile(r"^\s*(v_pk_(?:add|mul|fma)_f32)\b", re.M)
LLVM = "/opt/rocm/lib/llvm/bin"


def _nopk_flags():
    mk = open(os.path.join(CSRC, "Makefile")).read()
    m = re.search(r"^NOPK := (.+)$", mk, re.M)
    assert m, "Makefile lost NOPK"
    assert re.search(r"^FLAGS := .*\$\(NOPK\)", mk, re.M), "NOPK is not in every kernel's FLAGS"
    return m.group(1).split()


def test_no_packed_fp32_in_any_kernel_source():
    """Every kernel source, compiled with the Makefile's NOPK flags, has no packed FP32 VALU
    (v_pk_add / mul / fma_f32).  In fz_logmel's FFT they gave wrong results in lanes 48-63 of a wave
    while decode step kernels shared the CU (the corrupted frames move with those
    lanes; without packed FP32 0 of ~100k batches); any kernel may share a CU with the featurizer, so
    none carries them."""
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    flags = _nopk_flags()
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))

    def isa(src):
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "k.s")
            subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-w", *flags,
                            "--cuda-device-only", "-S", os.path.basename(src), "-o", out],
                           check=True, cwd=CSRC, capture_output=True)
            return open(out).read()

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        isas = dict(zip(srcs, ex.map(isa, srcs)))
    assert "fz_logmel_kernel" in isas[os.path.join(CSRC, "featurizer.hip")]
    bad = {os.path.basename(s): sorted(set(PACKED_FP32.findall(t))) for s, t in isas.items()}
    bad = {k: v for k, v in bad.items() if v}
    assert not bad, f"packed FP32 in kernel ISA: {bad}"
    # the flag is what removes them: without it the decoder has some (so the check can fail)
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "d.s")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-w",
                        "--cuda-device-only", "-S", "decoder.hip", "-o", out], check=True, cwd=CSRC, capture_output=True)
        assert PACKED_FP32.search(open(out).read())


def test_no_packed_fp32_in_built_objects():
    """The objects linked into librnnt_mi355x.so (what ships to the GPU box) carry no packed FP32:
    each object's gfx950 code object is unbundled from .hip_fatbin and disassembled."""
    objs = sorted(o for o in glob.glob(os.path.join(CSRC, "*.o"))
                  if os.path.exists(os.path.splitext(o)[0] + ".hip"))  # kernel objects (crash_report.o is host code)
    if not objs or not os.path.exists(os.path.join(LLVM, "clang-offload-bundler")):
        pytest.skip("library not built here")
    srcs = {os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(CSRC, "*.hip"))}
    assert srcs <= {os.path.splitext(os.path.basename(p))[0] for p in objs}, "some kernel objects are not built"
    bad = {}
    with tempfile.TemporaryDirectory() as td:
        for o in objs:
            b, co = os.path.join(td, "x.bundle"), os.path.join(td, "x.co")
            subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={b}", o], check=True, capture_output=True)
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={b}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", co], check=True, capture_output=True,
                                 text=True).stdout
            assert "s_endpgm" in dis
            hits = sorted(set(re.findall(r"\b(v_pk_(?:add|mul|fma)_f32)\b", dis)))
            if hits:
                bad[os.path.basename(o)] = hits
    assert not bad, f"packed FP32 in built objects (rebuild: make -C {CSRC}): {bad}"


def _kernel_resources(obj):
    """{kernel name: {agpr_count, vgpr_count, group_segment_fixed_size, private_segment_fixed_size}}
    from the AMDGPU metadata note of an object's gfx950 code object."""
    with tempfile.TemporaryDirectory() as td:
        b, co = os.path.join(td, "x.bundle"), os.path.join(td, "x.co")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={b}", obj], check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={b}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                               text=True).stdout
    out = {}
    for blk in re.split(r"\n  - (?=\.agpr_count:)", notes)[1:]:
        name = re.search(r"^    \.name:\s+(\S+)", blk, re.M)
        if not name:
            continue
        out[name.group(1)] = {k: int(re.search(rf"^\s*\.{k}:\s+(\d+)", blk, re.M).group(1))
                              for k in ("agpr_count", "vgpr_count", "group_segment_fixed_size",
                                        "private_segment_fixed_size")}
    return out


def test_coresident_decode_kernels_fit_beside_a_tick():
    """The decode step kernels the engine launches (decoder.hip SLIM_BOUNDS) must fit on a CU beside a
    256x256 encoder tick workgroup, or every decode launch waits for ticks to give up CUs again
    (MEASUREMENTS section 9).  Budget per CU: 160 KiB of LDS minus the tick's
    147456 B (TileCfg<4, 8, 2>::SMEM: two 64 KiB stages + the 16 KiB sigma table, dynamic LDS), and per
    SIMD 512 VGPRs minus the tick's two waves (8-VGPR granules, AGPRs included); no scratch."""
    objs = {n: os.path.join(CSRC, n + ".o") for n in ("encoder", "decoder")}
    if not all(os.path.exists(o) for o in objs.values()) or not os.path.exists(os.path.join(LLVM, "clang-offload-bundler")):
        pytest.skip("library not built here")
    enc, dec = _kernel_resources(objs["encoder"]), _kernel_resources(objs["decoder"])
    alloc = lambda r: -(-(r["vgpr_count"] + r["agpr_count"]) // 8) * 8  # noqa: E731
    tick = [r for n, r in enc.items() if "lstm_i8_tick_kernel" in n and "ILi4ELi8ELi2E" in n]
    assert len(tick) == 1, sorted(enc)
    tick_lds, tick_vgprs = 147456, 2 * alloc(tick[0])
    slim = {n: r for n, r in dec.items() if "_slim_kernel" in n}
    for want in ("dec_pred0h_slim_kernel", "dec_pred1x_slim_kernel", "dec_g_slim_kernel", "dec_joint_slim_kernel"):
        assert any(want in n for n in slim), (want, sorted(dec))
    for n, r in slim.items():
        assert r["group_segment_fixed_size"] + tick_lds <= 160 * 1024, (n, r)
        assert alloc(r) + tick_vgprs <= 512, (n, r, tick[0])
        assert r["private_segment_fixed_size"] == 0, (n, r)
    # the check can fail: the big-tile layer-1 step kernel does not fit (43 KiB of LDS, 218 VGPRs)
    big = [r for n, r in dec.items() if "dec_pred_kernelILi1E" in n]
    assert big and (big[0]["group_segment_fixed_size"] + tick_lds > 160 * 1024 or alloc(big[0]) + tick_vgprs > 512)
