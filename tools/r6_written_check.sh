#!/bin/bash
# round 6: the score keys' written mark -- the allreduce test, the in-process multi tests (shared
# k_score_keys, lo > 0 on one device) and the score tests
set -u
cd "$(dirname "$0")/.."
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "allreduce or multi or score or parity_bar" 2>&1 | tail -5
