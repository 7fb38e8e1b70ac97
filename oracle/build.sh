#!/bin/bash
# Build the oracle's C helpers (test infrastructure): liboracle_csrmv.so next
# to this script. Called by __graft_entry__.build(); the .so is git-ignored
# and travels to the GPU box with the tree.
set -e
cd "$(dirname "$0")"
gcc -O2 -fopenmp -ffp-contract=off -fPIC -shared -o liboracle_csrmv.so csrmv.c
