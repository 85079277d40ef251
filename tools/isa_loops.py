"""Per-basic-block instruction mix of one kernel in a hipcc -S listing, with the
blocks that end in a backward branch (loops) marked.  Usage:
    python3 tools/isa_loops.py build/trace_kernel.s <mangled-name-substring> [min_insts]"""
import re
import sys

path, pat = sys.argv[1], sys.argv[2]
min_n = int(sys.argv[3]) if len(sys.argv) > 3 else 8
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(pat) + r"\S*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.section") or re.match(r"^\.Lfunc_end", lines[i]))
body = lines[start:end]
blocks, cur, order = {}, None, []
for l in body:
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        cur = m.group(1); blocks[cur] = []; order.append(cur); continue
    s = l.strip()
    if not s or s.startswith((";", ".", "//")) or cur is None:
        continue
    blocks[cur].append(s.split()[0])
pos = {b: i for i, b in enumerate(order)}
for b in order:
    ins = blocks[b]
    if len(ins) < min_n:
        continue
    kinds = {}
    for op in ins:
        k = ("v_" + ("f64" if "f64" in op else "f16" if ("f16" in op or "mix" in op) else "other")) if op.startswith("v_") else \
            "s_" if op.startswith("s_") else "ds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "flat_", "buffer_", "scratch_")) else op
        kinds[k] = kinds.get(k, 0) + 1
    back = ""
    for l2 in body:
        pass
    tgt = [re.search(r"(\.LBB\S+)", x) for x in []]
    print(f"{b}: {len(ins)} insts {dict(sorted(kinds.items()))}")
