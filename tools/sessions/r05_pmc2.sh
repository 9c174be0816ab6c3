#!/bin/bash
# round 5: per-K PMC, two K per call:  bash tools/sessions/r05_pmc2.sh <K1> <K2>
set -u
cd "${GRAFT_REPO_ROOT:-.}"
bash tools/sessions/r05_pmc.sh $1 && bash tools/sessions/r05_pmc.sh $2
