# Per-step kernel summary from a rocprofv3 --kernel-trace SQLite database:
#   python scripts/rocpd_step_summary.py run_results.db <kernel name marking one step> <steps> [end]
# The marker is the first kernel of a step, or with "end" its last (e.g. finalize_kernel):
# the window is then the nsteps steps that end at the last nsteps markers.
import sqlite3, sys, re, collections
db, marker, nsteps = sys.argv[1], sys.argv[2], int(sys.argv[3])
c = sqlite3.connect(db)
rows = list(c.execute("select name, start, end from kernels order by start"))
idx = [i for i, r in enumerate(rows) if marker in r[0]]
if len(sys.argv) > 4 and sys.argv[4] == "end":
    sel = rows[idx[len(idx) - nsteps - 1] + 1: idx[-1] + 1]
else:
    sel = rows[idx[len(idx) - nsteps]:]
span = (sel[-1][2] - sel[0][1]) / 1e3 / nsteps
agg = collections.defaultdict(lambda: [0, 0.0])
for n, s, e in sel:
    short = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))[:110]
    agg[short][0] += 1; agg[short][1] += (e - s) / 1e3
tot = sum(v[1] for v in agg.values()) / nsteps
print(f"per step: wall span {span:.1f} us, kernel busy {tot:.1f} us, {len(sel)/nsteps:.1f} launches")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t/nsteps:9.2f} us  {n/nsteps:5.2f}x  {k}")
