#!/bin/bash
# Round 6, call t: issue priority in the product scan (diagnostic library,
# LMI_SCAN_ABL 80: s_setprio 1 around each wave's MFMA stream; 81: the late
# waves at priority 1; 82: the early ones; 83: none, the baseline with the same diagnostic clocks), lists checked bitwise against abl 0.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp
mkdir -p gpurun_out
LMI_LIB_NAME=liblmi_hip_abl.so timeout -k 10 600 python -u tools/prof_scan.py --abl 83,80,82,83,80,82,0 --reps 10 --check \
  > gpurun_out/r6t_prio.txt 2>&1
rc=$?; grep -v "^\s*$" gpurun_out/r6t_prio.txt | tail -30; exit $rc
