#!/bin/bash
set -o pipefail
bash scripts/r05/check2.sh && bash scripts/r05/tsweep.sh
