#!/bin/bash
set -o pipefail
bash scripts/r3_ab_lag.sh ${1:-lag} && bash scripts/r3_suite.sh
