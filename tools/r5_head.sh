#!/bin/bash
# round 5: the loss head's path (1/mb from the host; wave 0's H1 plane stores
# after the head): bitwise + in-graph step against the last commit, then the
# phase stamps of the probe build
set -o pipefail
mkdir -p gpurun_out
TAG=r5hd BITS=1 VNAME=head bash tools/ab_head.sh &&
PROBE_H=256 PROBE_CHAIN=1 timeout -k 10 120 python3 tools/phase_probe.py probe > gpurun_out/r5hd_phase.txt 2>&1
