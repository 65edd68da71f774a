#!/bin/bash
# Round 4: kgx_dense cost decomposition at C5's shape (2.45M x (100+100) -> 100,
# ReLU): full / no MFMA / no stores / no loads + split (KGX_DENSE_DEBUG 0/1/2/4,
# experiment build), to see what bounds the 0.75 ms.
# Build first (here): make -C keras-geometric_amd/csrc variant NAME=exp DEFS=-DKGX_EXPERIMENTS
set -o pipefail
mkdir -p gpurun_out/r4dc5
export TMPDIR=/tmp
O=gpurun_out/r4dc5
V=keras-geometric_amd/lib/variants/libkgx_exp.so
for d in 0 1 2 4 3 0; do
  KGX_LIB=$V KGX_DENSE_DEBUG=$d timeout -k 10 300 python tools/bench_dense.py --only C5,C4 --reps 30 > $O/dense_dbg$d.jsonl 2>> $O/err.log || exit $?
done
