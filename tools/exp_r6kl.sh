#!/bin/bash
# round 6: r6k (stream pieces by partitions per GPU) then r6l (the fix-up's lane pass)
set -o pipefail
cd "$(dirname "$0")/.."
tools/exp_r6k.sh && tools/exp_r6l.sh
