"""Per-kernel VGPR / AGPR / scratch / occupancy table from a hipcc -Rpass-analysis=kernel-resource-usage
log: python scripts/kernel_resources.py LOG [name-filter]. Flags kernels with scratch (stack objects
or spills), which on these kernels means a lambda was not inlined or a register array went to memory."""
import re
import sys

cur, info, rows = None, {}, []
for line in open(sys.argv[1]):
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        if cur:
            rows.append((cur, info))
        cur, info = m.group(1), {}
        continue
    m = re.search(r'remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill): (\d+)', line)
    if m and cur:
        info[m.group(1).replace(' [bytes/lane]', '').replace(' [waves/SIMD]', '')] = int(m.group(2))
if cur:
    rows.append((cur, info))
flt = sys.argv[2] if len(sys.argv) > 2 else ''
bad = 0
for n, i in rows:
    if flt in n:
        flag = ' <-- SCRATCH' if i.get('ScratchSize', 0) else ''
        bad += bool(flag)
        print(f"{i.get('VGPRs', '?'):>4} v {i.get('AGPRs', '?'):>4} a {i.get('ScratchSize', '?'):>5} scr "
              f"{i.get('VGPRs Spill', '?'):>4} spill occ {i.get('Occupancy', '?')}  {n[:100]}{flag}")
print(f'{len(rows)} kernels, {bad} with scratch')
