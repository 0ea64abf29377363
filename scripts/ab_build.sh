#!/bin/bash
# build libkmeans_amd_new.so (working tree) and libkmeans_amd_prev.so (HEAD)
# for scripts/gpu_ablib.sh; leaves the working tree's build as the product
set -e
cd "$(dirname "$0")/.."
P=assignment--2-group7-distributed-k-means_amd
make -s -C $P/csrc >/dev/null
cp $P/libkmeans_amd.so $P/libkmeans_amd_new.so
git stash -q
trap 'git stash pop -q' EXIT
make -s -C $P/csrc >/dev/null
cp $P/libkmeans_amd.so $P/libkmeans_amd_prev.so
git stash pop -q
trap - EXIT
make -s -C $P/csrc >/dev/null
