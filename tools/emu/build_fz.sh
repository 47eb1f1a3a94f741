#!/bin/bash
# Development: build the host emulation of the featurizer kernels (tools/emu/fz_emu.cpp) with
# AddressSanitizer into build_dev/emu_fz/.  featurizer.hip is copied with its GPU-only constructs
# rewritten for the host: the LDS wait before a wave hand-off is dropped (the wave barrier that
# follows it is emulated), __shared__ arrays become statics that lane 0 poisons at workgroup start.
set -e
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
SRC=${EMU_SRC:-$ROOT/rnnt-inference_amd/csrc}
OUT=${EMU_OUT:-$ROOT/build_dev/emu_fz}
mkdir -p $OUT
python3 - "$SRC" "$OUT" "$ROOT" <<'PY'
import sys
src, out, root = sys.argv[1:4]
t = open(f"{src}/featurizer.hip").read()
t = t.replace('asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");', '')
t = t.replace('#include "../../include/rnnt_mi355x.h"', f'#include "{root}/include/rnnt_mi355x.h"')
anchor = '  float2(*scr)[4][SCR] = scrs[sub];\n'
assert anchor in t, "fz_logmel_kernel LDS declarations moved: update tools/emu/build_fz.sh"
t = t.replace(anchor, anchor + '  if (threadIdx.x == 0) { emu_fz_poison(tab, sizeof(tab)); emu_fz_poison(win, sizeof(win)); '
              'emu_fz_poison(segs, sizeof(segs)); emu_fz_poison(scrs, sizeof(scrs)); }\n')
if 'asm volatile' in t or 'asm(' in t:
    raise SystemExit('unhandled asm in featurizer.hip')
open(f"{out}/featurizer_emu.hip.cpp", "w").write(t)
for name in ("rnnt_device.hpp", "featurizer.hpp"):
    open(f"{out}/{name}", "w").write(open(f"{src}/{name}").read())
PY
CXX=/opt/rocm/lib/llvm/bin/clang++
if [ "${EMU_ASAN:-1}" = 1 ]; then SAN="-O1 -fsanitize=address -fno-omit-frame-pointer"; else SAN="-O2"; fi
$CXX $SAN -g -std=c++20 -ffp-contract=off -pthread -I$ROOT/tools/emu -I$OUT $ROOT/tools/emu/fz_emu.cpp -o $OUT/fz_emu -lm
echo "built $OUT/fz_emu"
