"""Scan a --save-temps gfx950 .s file for vector-memory ops whose result is
waited on soon after issue (a linear, branch-unaware approximation of the
vmcnt queue: gfx9 counts loads and stores in one in-order counter).
    python3 tools/isa_waits.py <file.s> [kernel-substring] [max-distance]
Prints, per kernel, each op retired by an s_waitcnt vmcnt(n) fewer than
max-distance (default 12) instructions after it was issued."""
import re
import sys

path = sys.argv[1]
want = sys.argv[2] if len(sys.argv) > 2 else ""
maxd = int(sys.argv[3]) if len(sys.argv) > 3 else 12
lines = open(path).read().split("\n")
kern = None
body = []


def scan(name, body):
    q = []  # (index, text) of outstanding vm ops, oldest first
    hits = []
    for i, l in enumerate(body):
        if re.match(r"(global|buffer|flat|scratch)_(load|store|atomic)", l):
            q.append((i, l))
            continue
        m = re.search(r"vmcnt\((\d+)\)", l)
        if m and l.startswith("s_waitcnt"):
            n = int(m.group(1))
            while len(q) > n:
                j, t = q.pop(0)
                if i - j < maxd and "store" not in t:
                    hits.append((j, i - j, t[:60], body[i + 1][:40] if i + 1 < len(body) else ""))
        if l.startswith("s_endpgm"):
            q = []
    print(f"{name[:40]}: {len(body)} instrs, {len(hits)} early waits")
    for j, d, t, nxt in hits:
        print(f"   @{j:5d} +{d:2d}  {t}  -> {nxt}")


for raw in lines:
    l = raw.strip()
    m = re.match(r"^(_Z\w+|k_\w+):", raw)
    if m:
        kern = m.group(1)
        body = []
        continue
    if kern is None or not l or l.startswith(";") or l.startswith("."):
        continue
    body.append(l)
    if l.startswith("s_endpgm"):
        if want in kern:
            scan(kern, body)
        kern = None
