"""Static instruction counts per engine phase (MTE_MARKERS build): for each MTE_PROF scope, the
instructions between its begin/end markers in one kernel's assembly, inclusive of nested scopes and
exclusive of them. Usage: python tools/asm_regions.py fluidframework_amd/_build/markers.s k_lds<false>"""
import re
import sys
from collections import Counter

NAMES = ["apply", "resolve", "insert_slot", "range", "zamboni", "scour", "heap", "find_seg", "map", "pack",
         "fetch", "lru", "text", "alloc", "ops", "total"]
# row engine (reg_engine.hpp RgProf, markers 100 + slot)
RG_NAMES = ["rg_total", "rg_fetch", "rg_apply", "rg_resolve", "rg_insert_slot", "rg_split", "rg_range", "rg_zamboni",
            "rg_scour", "rg_heap", "rg_find_seg", "rg_pack", "rg_lru", "rg_ops", "rg_n_resolve", "rg_n_scour",
            "rg_n_scour_changed", "rg_n_pack", "rg_n_pop", "rg_n_split_blk", "rg_n_move", "rg_split_at", "rg_ins",
            "rg_rem", "rg_msn", "rg_zam_edit"]


def name(s):
    if s >= 100 and s - 100 < len(RG_NAMES):
        return RG_NAMES[s - 100]
    return NAMES[s] if s < len(NAMES) else str(s)
path = sys.argv[1]
kernel = sys.argv[2] if len(sys.argv) > 2 else "k_lds<false>"
mangled = {"k_lds<false>": "_ZN3mte5k_ldsILb0ELi0EEEvNS_6ParamsE", "k_solo<false>": "_ZN3mte6k_soloILb0ELi0EEEvNS_6ParamsE", "k_hbmq<false>": "_ZN3mte6k_hbmqILb0ELi0EEEvNS_6ParamsE"}[kernel]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(mangled + ":"))
end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i] and i > start)
incl, excl, kinds = Counter(), Counter(), {}
stack = []
ins = re.compile(r"^\s+([sv]_|ds_|global_|scratch_|buffer_|flat_)([a-z0-9_]+)")
total = 0
for l in lines[start:end + 1]:
    m = re.search(r"MTE_BEGIN (0x[0-9a-fA-F]+|\d+)", l)
    if m:
        stack.append(int(m.group(1), 0))
        continue
    m = re.search(r"MTE_END (0x[0-9a-fA-F]+|\d+)", l)
    if m:
        if stack and stack[-1] == int(m.group(1), 0):
            stack.pop()
        continue
    if ins.match(l):
        total += 1
        for s in set(stack):
            incl[s] += 1
        if stack:
            excl[stack[-1]] += 1
            kinds.setdefault(stack[-1], Counter())[ins.match(l).group(1)] += 1
print(f"{kernel}: {total} instructions")
for s in sorted(incl, key=lambda x: -incl[x]):
    k = kinds.get(s, Counter())
    print(f"{name(s):16s} incl {incl[s]:6d} excl {excl[s]:6d}  "
          + " ".join(f"{a}{b}" for a, b in sorted(k.items(), key=lambda x: -x[1])[:5]))
