#!/bin/bash
# round 5: dynamic LDS, registers and resident workgroups per CU of every
# chain launch the r05g tuner chose at batch 24, with its launch time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05am
mkdir -p $O
timeout -k 10 300 python -u tools/chain_occupancy.py --tune tools/sessions/r05am_tune_r05g.txt --resources profiles/r05am_chain_resources.tsv > $O/chain_occupancy_b24.txt 2>&1 || exit 1
echo done
