#!/bin/bash
set -o pipefail
GO2PI_W8=1 timeout -k 10 120 python3 tools/w8_debug.py && timeout -k 10 120 python3 tools/w8_debug.py
