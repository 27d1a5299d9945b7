"""Instruction mix of a kernel's loops, from hipcc -S output (gfx950).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc -S --offload-device-only \
        csrc/assign_mfma.hip -o /tmp/a.s
    python tools/isa_loop_mix.py /tmp/a.s 'ring3_kernelILi128ELi8ELi2ELi4ELi4ELb0E'

For every loop of the first kernel whose symbol contains the pattern (a loop = the lines
from a ``Loop Header`` label to the last back-branch to it), prints the count per class:
MFMA, VALU (and the top opcodes), LDS (ds_*), VMEM / LDS-DMA, SALU, s_waitcnt, s_nop,
s_barrier; plus VALU per MFMA.  Used for the issue-budget attributions in
docs/PERF_NOTES.md (counts are static: per loop trip, not weighted by execution)."""
import re
import sys
from collections import Counter


def kernel_body(lines, pat):
    for i, l in enumerate(lines):
        sym = l.split(":")[0]
        if l.startswith("_Z") and pat in sym and re.match(r"^\S+:(\s|$)", l):
            for j in range(i, len(lines)):
                if lines[j].startswith(".Lfunc_end"):
                    return lines[i:j]
    raise SystemExit(f"no kernel matching {pat}")


def classify(op):
    if "mfma" in op:
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op == "s_waitcnt":
        return "waitcnt"
    if op == "s_nop":
        return "nop"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    body = kernel_body(open(path).read().split("\n"), pat)
    # basic blocks: a label line (".LBBx_y:" or "; %bb.N:") opens one; the compiler's
    # comment on it names the loop it belongs to ("Loop Header: Depth=d" on the header,
    # "in Loop: Header=BBx_y Depth=d" on the others)
    loops = {}
    cur = None
    for l in body:
        m = re.match(r"^(\.LBB(\w+)|; %bb\.\d+):", l)
        if m:
            cur = None
            h = re.search(r"Header=BB(\w+) Depth=(\d+)", l)
            if h:
                cur = (h.group(1), int(h.group(2)))
            elif "Loop Header" in l and m.group(2):
                d = re.search(r"Depth=(\d+)", l)
                cur = (m.group(2), int(d.group(1)) if d else 1)
            continue
        if cur is None:
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        loops.setdefault(cur, Counter())[t.split()[0]] += 1
    for (lab, depth), ops in loops.items():
        cls = Counter()
        for op, n in ops.items():
            cls[classify(op)] += n
        mf = max(1, cls["mfma"])
        print(f"loop BB{lab} depth {depth}: " + ", ".join(f"{k} {v}" for k, v in sorted(cls.items())))
        print(f"  VALU per MFMA {cls['valu'] / mf:.2f}; top VALU: " + ", ".join(
            f"{k} {v}" for k, v in ops.most_common() if k.startswith("v_") and "mfma" not in k)[:500])
        print("  SALU: " + ", ".join(f"{k} {v}" for k, v in ops.most_common()
                                     if classify(k) == "salu")[:300])


if __name__ == "__main__":
    main()
