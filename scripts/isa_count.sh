#!/usr/bin/env bash
# Static VALU / total instruction counts per device function (scripts/isa_count.hip), gfx950.
set -eu
cd "$(dirname "$0")"
mkdir -p ../build_variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off --cuda-device-only -S \
    isa_count.hip -o ../build_variants/isa_count.s
python3 - ../build_variants/isa_count.s <<'EOF'
import re, sys
cur, stats = None, {}
for line in open(sys.argv[1]):
    m = re.match(r"^(k_\w+):", line)
    if m:
        cur = m.group(1); stats[cur] = [0, 0, 0, 0]; continue
    if cur and line.startswith("\t.size"):
        cur = None; continue
    if cur:
        s = line.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        op = s.split()[0]
        st = stats[cur]
        st[0] += 1
        if op.startswith("v_"): st[1] += 1
        if "f64" in op: st[2] += 1
        if op.startswith("s_cbranch") or op.startswith("s_branch"): st[3] += 1
print(f"{'kernel':24s} {'total':>6s} {'valu':>6s} {'f64':>6s} {'branch':>6s}")
for k, (t, v, f, b) in stats.items():
    print(f"{k:24s} {t:6d} {v:6d} {f:6d} {b:6d}")
EOF
