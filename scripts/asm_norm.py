"""Normalised device assembly (instructions + labels, no comments / directives / metadata), for checking
that a source refactor (e.g. pruning a compile-time knob's dead arm) leaves the code object unchanged.
usage: python scripts/asm_norm.py a.s [b.s]   -- prints a digest per function, or diffs two files"""
import hashlib
import re
import sys


def functions(path):
    out, cur = {}, None
    for line in open(path):
        m = re.match(r"^([A-Za-z_][\w.$]*):", line)
        if m and not m.group(1).startswith(".L"):
            cur = m.group(1)
            out[cur] = []
            continue
        if cur is None:
            continue
        s = line.split(";")[0].strip()
        if not s or s.startswith((".", "//")):
            if line.startswith("\t.size") or line.startswith(".Lfunc_end"):
                cur = cur
            continue
        out[cur].append(s)
    return {k: v for k, v in out.items() if v}


def main():
    a = functions(sys.argv[1])
    if len(sys.argv) == 2:
        for k, v in a.items():
            print(hashlib.sha1("\n".join(v).encode()).hexdigest()[:12], len(v), k)
        return
    b = functions(sys.argv[2])
    diff = 0
    for k in sorted(set(a) | set(b)):
        if a.get(k) != b.get(k):
            diff += 1
            print("DIFF", k, len(a.get(k, [])), len(b.get(k, [])))
    print("functions:", len(a), len(b), "differing:", diff)
    sys.exit(1 if diff else 0)


if __name__ == "__main__":
    main()
