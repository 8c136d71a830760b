#!/bin/bash
# r05 combined A/B pass: the 8-wave lean kernel (tools/r05_w8.sh), then the lean
# controller tick (tools/r05_ctl_ab.sh).
set -o pipefail
bash tools/r05_w8.sh && bash tools/r05_ctl_ab.sh
