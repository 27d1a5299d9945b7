#!/usr/bin/env python3
"""Audit a hipcc .s: no instruction may read or write the destination VGPRs of an inline-asm
global_load (between ;;#ASMSTART/;;#ASMEND) before the next explicit s_waitcnt vmcnt(0)."""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def main(path):
    lines = open(path).read().splitlines()
    bad = 0
    pending = {}
    in_asm = False
    for i, l in enumerate(lines):
        s = l.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith(";") or s.endswith(":"):
            continue
        if in_asm and s.startswith("global_load"):
            dst = s.split()[1].rstrip(",")
            for r in regs(dst):
                pending[r] = i
            continue
        if in_asm and "s_waitcnt vmcnt(0)" in s:
            pending.clear()
            continue
        ops = re.findall(r"v\[\d+:\d+\]|v\d+\b", s)
        touched = set().union(*[regs(o) for o in ops]) if ops else set()
        hit = touched & set(pending)
        if hit:
            bad += 1
            print(f"line {i+1}: touches in-flight asm-load regs {sorted(hit)}: {s}")
    print("asm-load audit:", "OK" if bad == 0 else f"{bad} violations")
    return bad


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1]) else 0)
