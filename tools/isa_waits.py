"""List the vector loads that are waited for at once (load, then s_waitcnt vmcnt(0)) per kernel,
by source line — each one a memory round trip of its own (the round-6 audit).

  cd kmerlsh_amd/csrc && hipcc --offload-arch=gfx950 -O3 <the Makefile's flags> -gline-tables-only \
      --cuda-device-only -S klsh_merge.hip -o /tmp/m.s
  python tools/isa_waits.py /tmp/m.s [top N] [kernel-name substring]

Without -gline-tables-only the source lines print as None.  Loads that must wait (a pointer
chase, a spin) show up too: read the line before changing it.
"""
import re
import sys
from collections import Counter


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    only = sys.argv[3] if len(sys.argv) > 3 else ""
    s = open(path).read()
    files = {m.group(1): m.group(2).split("/")[-1]
             for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', s, re.M)}
    files.update({m.group(1): m.group(2).split("/")[-1]
                  for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]+)"\s*$', s, re.M)})
    rows = []
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        if only and only not in m.group(1):
            continue
        end = s.find(".Lfunc_end", m.start())
        loc, body = None, []
        for ln in s[m.start():end].split("\n"):
            t = ln.strip()
            if t.startswith(".loc"):
                p = t.split()
                loc = f"{files.get(p[1], p[1])}:{p[2]}"
                continue
            if not t or t.startswith((";", ".")) or t.endswith(":"):
                continue
            body.append((t, loc))
        c = Counter(loc for i, (t, loc) in enumerate(body[:-1])
                    if re.match(r"(global|buffer|flat)_load", t)
                    and body[i + 1][0].startswith("s_waitcnt") and "vmcnt(0)" in body[i + 1][0])
        if c:
            rows.append((sum(c.values()), m.group(1), c.most_common(5)))
    for n, name, where in sorted(rows, reverse=True)[:top]:
        print(f"{n:4d}  {name[:90]}")
        for loc, k in where:
            print(f"        {k:3d} at {loc}")


if __name__ == "__main__":
    main()
