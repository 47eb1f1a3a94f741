#!/bin/bash
# Development: build the host emulation of the decode kernels (tools/emu/dec_emu.cpp) with
# AddressSanitizer into build_dev/emu/.  The sources are copied with the few GPU-only constructs
# (s_barrier asm, dynamic LDS, address-space typedefs) rewritten for the host.
set -e
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
SRC=${EMU_SRC:-$ROOT/rnnt-inference_amd/csrc}
OUT=${EMU_OUT:-$ROOT/build_dev/emu}
mkdir -p $OUT
python3 - "$SRC" "$OUT" <<'PY'
import re, sys
src, out = sys.argv[1], sys.argv[2]
def fix(text):
    text = text.replace('asm volatile("s_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory")', 'emu_sync()')
    text = text.replace('asm volatile("s_waitcnt vmcnt(0)\\n\\ts_waitcnt lgkmcnt(0)\\n\\ts_barrier" ::: "memory")', 'emu_sync()')
    text = text.replace('asm volatile("" : "+v"(c));', '')
    text = text.replace('asm volatile("s_waitcnt vmcnt(0)" ::: "memory");', '')  # persistent decode (not emulated)
    text = text.replace('asm("v_and_b32 %0, 0xffffff, %1" : "=v"(r) : "v"(e));', 'r = e & 0xffffff;')
    text = re.sub(r'extern __shared__ (__attribute__\(\(aligned\(16\)\)\) )?(\w+) (\w+)\[\];',
                  r'static \1\2 \3[1 << 17];', text)
    text = re.sub(r'__attribute__\(\(address_space\(\d\)\)\) ', '', text)
    if 'asm volatile' in text or 'asm(' in text:
        raise SystemExit('unhandled asm in ' + text[:40])
    return text
for name, dst in (("decoder.hip", "decoder_emu.hip.cpp"), ("rnnt_device.hpp", "rnnt_device.hpp"), ("decoder.hpp", "decoder.hpp")):
    open(f"{out}/{dst}", "w").write(fix(open(f"{src}/{name}").read()))
PY
CXX=/opt/rocm/lib/llvm/bin/clang++
# EMU_ASAN=0: an optimised build without AddressSanitizer (the CPU test's build)
if [ "${EMU_ASAN:-1}" = 1 ]; then SAN="-O1 -fsanitize=address -fno-omit-frame-pointer"; else SAN="-O2"; fi
# features of the decoder being emulated (the harness adapts to either step structure)
FEAT=""
grep -q "g_dec_err" $SRC/decoder.hip && FEAT="$FEAT -DEMU_HAS_DEC_CHECK"
grep -q "float\* ah0;" $SRC/decoder.hpp && FEAT="$FEAT -DEMU_HAS_AH"
$CXX $SAN -g -std=c++20 -ffp-contract=off -pthread $FEAT \
  -DRNNT_DEC_CHECK -DRNNT_EMU ${EMU_CFLAGS} -I$ROOT/tools/emu -I$OUT $ROOT/tools/emu/dec_emu.cpp $ROOT/oracle/rnnt_oracle.c \
  -o $OUT/dec_emu -lm
echo "built $OUT/dec_emu"
