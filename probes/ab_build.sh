#!/bin/bash
# Builds an alternative libofx_spmm.so of the same sources with extra compile flags, for A/B
# timing through OFX_SPMM_LIB (of-spmm_amd/oneflow_spmm/_lib.py).
# usage: probes/ab_build.sh <tag> "<-DKNOB=value ...>"   ->  of-spmm_amd/oneflow_spmm/libofx_spmm_<tag>.so
set -eu
cd "$(dirname "$0")/../of-spmm_amd"
make -s -j8 BUILD=build_$1 OUT=oneflow_spmm/libofx_spmm_$1.so EXTRA="$2"
