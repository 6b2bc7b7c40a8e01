#!/bin/bash
set -o pipefail
bash scripts/r05/ab_flush.sh && SWEEP=1 bash scripts/r05/suite.sh
