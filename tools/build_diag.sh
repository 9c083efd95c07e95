#!/bin/bash
# Diagnostic variants of libfattn.so (never loaded by the product path; bench.py / tools
# select one with FATTN_LIB=<name>): each drops one phase of the split kernel so the
# phases' costs can be read off the un-instrumented kernel's time.
set -e
cd "$(dirname "$0")/.."
SRC=$(ls ggml-cuda-experiments_amd/csrc/*.hip)
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -Iinclude -shared"
build() { /opt/rocm/bin/hipcc $F "${@:2}" $SRC -o ggml-cuda-experiments_amd/lib/libfattn_diag_$1.so; }
build nocompute -DFATTN_DIAG_NOCOMPUTE &
build notail -DFATTN_DIAG_NOTAIL &
build dmaonly -DFATTN_DIAG_NOCOMPUTE -DFATTN_DIAG_NOTAIL &
build nopublish -DFATTN_DIAG_NOPUBLISH &
wait
build noatomic -DFATTN_DIAG_NOATOMIC &
build nomem -DFATTN_DIAG_NOMEM &
build nomem_notail -DFATTN_DIAG_NOMEM -DFATTN_DIAG_NOTAIL &
wait
