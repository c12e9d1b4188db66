#!/usr/bin/env python3
"""Compact register / LDS / spill table from `make asm` remarks (kernel-resource-usage).
usage: make -C nanopore-barcoding-orc_amd asm 2> log; python tools/kres.py log [substring ...]"""
import re
import sys

cur, rows = None, {}
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"\s(VGPRs|VGPRs Spill|SGPRs Spill|TotalSGPRs|AGPRs|ScratchSize \[bytes/lane\]|"
                  r"LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
keys = sys.argv[2:]
for k, v in rows.items():
    if keys and not any(s in k for s in keys):
        continue
    print(f"{k[:60]:60s} vgpr {v.get('VGPRs')} spill {v.get('VGPRs Spill')} "
          f"sspill {v.get('SGPRs Spill')} scratch {v.get('ScratchSize [bytes/lane]')} "
          f"lds {v.get('LDS Size [bytes/block]')} occ {v.get('Occupancy [waves/SIMD]')}")
