#!/bin/bash
# Builds a variant of the library with a generator switch of mythril_amd/csrc/gen_asm_core.py
# flipped, beside the default one, for on-box A/B runs (MYTHRIL_HIP_LIB=<variant .so>):
#   bash scripts/build_variant.sh nopf MH_GEN_LV_PREFETCH=0
# -> mythril_amd/libmythril_hip_nopf.so (the default library and asm_core.inc are left as built).
set -e
NAME=${1:?name}
shift
cd "$(dirname "$0")/../mythril_amd/csrc"
trap 'python3 gen_asm_core.py > asm_core.inc' EXIT
env "$@" python3 gen_asm_core.py > asm_core.inc
make -s -j8 OUT=../libmythril_hip_$NAME.so OBJDIR=../../build/csrc_$NAME
