#!/bin/bash
# GPU box: A/B of engine builds on C2 and C3 (tools/ab_cfg.sh), variants as arguments.
set -e
CFG=C2 REPS=4 bash tools/ab_cfg.sh "$@"
CFG=C3 REPS=2 bash tools/ab_cfg.sh "$@"
