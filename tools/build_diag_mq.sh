#!/bin/bash
# Diagnostic variants of the multi-query kernel (never loaded by the product
# path; select with FATTN_LIB=<name>): each drops one phase so its cost can be
# read off the un-instrumented kernel's time.
set -e
cd "$(dirname "$0")/.."
SRC=$(ls ggml-cuda-experiments_amd/csrc/*.hip)
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -Iinclude -shared"
build() { /opt/rocm/bin/hipcc $F "${@:2}" $SRC -o ggml-cuda-experiments_amd/lib/libfattn_diag_$1.so; }
build mq_nomem -DFATTN_MQ_NOMEM &
build mq_nodeq -DFATTN_MQ_NODEQ &
build mq_nocompute -DFATTN_MQ_NOCOMPUTE &
build mq_dmaonly -DFATTN_MQ_NOCOMPUTE -DFATTN_MQ_NODEQ &
wait
