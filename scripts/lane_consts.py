"""Debug: which values the compiler keeps in VGPR lanes (SGPR spills) and how often they are read
back (v_readlane), from a device assembly listing of one kernel.  usage: lane_consts.py <kernel.s>"""
import re, sys, collections, struct
L = open(sys.argv[1]).read().split('\n')
lit, wl = {}, {}
for l in L:
    s = l.strip()
    m = re.match(r's_mov_b32 (s\d+), (0x[0-9a-f]+|-?\d+)', s)
    if m:
        lit[m.group(1)] = int(m.group(2), 0) & 0xffffffff
        continue
    m = re.match(r'v_writelane_b32 (v\d+), (s\d+), (\d+)', s)
    if m:
        wl[(m.group(1), int(m.group(3)))] = lit.get(m.group(2))
c = collections.Counter()
for l in L:
    m = re.match(r'\s*v_readlane_b32 (s\d+), (v\d+), (\d+)', l)
    if m:
        c[(m.group(2), int(m.group(3)))] += 1
print("reads", sum(c.values()))
for (v, ln), n in c.most_common(40):
    lo, hi = wl.get((v, ln)), wl.get((v, ln + 1))
    val = ''
    if lo is not None and hi is not None:
        val = struct.unpack('<d', struct.pack('<II', lo, hi))[0]
    print(f"{v}:{ln:3d} reads {n:4d}  lo {lo if lo is None else hex(lo)}  as double(lo,hi) {val}")
