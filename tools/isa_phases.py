"""Per-phase static instruction counts of a kernel compiled with phase markers.

    python tools/isa_phases.py FILE.s KERNEL_SYMBOL_PREFIX

A diagnostic copy of a kernel gets `asm volatile("; PHASE_<name>")` markers fenced by
`__builtin_amdgcn_sched_barrier(0)` between its phases; this prints the VALU / LDS / memory
instruction counts between consecutive markers (DESIGN.md per-phase VALU budgets).
"""
import collections
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_stats import classify  # noqa: E402

path, prefix = sys.argv[1], sys.argv[2]
phase = "prologue"
cnt = collections.defaultdict(collections.Counter)
inside = False
order = []
for ln in open(path).read().splitlines():
    if ln.startswith(prefix):
        inside = True
        order.append(phase)
        continue
    if inside and ln.startswith(".Lfunc_end"):
        break
    if not inside:
        continue
    m = re.search(r"; PHASE_(\w+)", ln)
    if m:
        phase = m.group(1)
        if phase not in order:
            order.append(phase)
        continue
    t = ln.strip()
    if not t or t.startswith((";", ".")) or t.endswith(":"):
        continue
    cnt[phase][classify(t.split()[0])] += 1
tot = 0
for ph in order:
    c = cnt[ph]
    valu = sum(c[k] for k in ("valu_f64", "valu_other", "valu_mov", "dpp", "lane_xfer"))
    tot += valu
    print(f"{ph:10s} VALU {valu:5d}  f64 {c['valu_f64']:4d} other {c['valu_other']:4d} mov {c['valu_mov']:4d} "
          f"dpp {c['dpp']:4d} xfer {c['lane_xfer']:3d} | lds {c['lds']} vmem {c['vmem_load']}+{c['vmem_store']} "
          f"salu {c['salu']}")
print("total VALU", tot)
