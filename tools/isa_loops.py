"""Per-basic-block instruction mix of one kernel in a hipcc -S listing, with the
blocks that a backward branch reaches (loop heads) and the branches that close
them marked.  Usage:
    python3 tools/isa_loops.py build/trace_kernel.s <mangled-name-substring> [min_insts] [--dump BLOCK ...]
Listing: hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S csrc/trace_kernel.hip (same flags as the
Makefile).  --dump prints the instructions of the named blocks (e.g. .LBB74_15)."""
import re
import sys

args = [a for a in sys.argv[1:]]
dump = []
if "--dump" in args:
    i = args.index("--dump")
    dump, args = args[i + 1:], args[:i]
path, pat = args[0], args[1]
min_n = int(args[2]) if len(args) > 2 else 8
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(pat) + r"\S*:", l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith("\t.section") or re.match(r"^\.Lfunc_end", lines[i]))
body = lines[start:end]
blocks, text, cur, order = {}, {}, "entry", ["entry"]
blocks[cur], text[cur] = [], []
for l in body[1:]:
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        cur = m.group(1); blocks[cur] = []; text[cur] = []; order.append(cur); continue
    s = l.strip()
    if not s or s.startswith((";", ".", "//")):
        continue
    blocks[cur].append(s.split()[0])
    text[cur].append(s.split(";")[0].rstrip())
pos = {b: i for i, b in enumerate(order)}
# back edges: a branch in block b to a block at or before b
heads = {}
for b in order:
    for t in text[b]:
        m = re.match(r"s_(c)?branch\S*\s+(\.LBB\S+)", t)
        if m and m.group(2) in pos and pos[m.group(2)] <= pos[b]:
            heads.setdefault(m.group(2), []).append(b)


def kind(op):
    if op.startswith("v_"):
        return "v_f64" if "f64" in op else "v_f16" if ("f16" in op or "mix" in op) else "v_other"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "s_"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith(("global_", "flat_", "buffer_", "scratch_")):
        return "vmem"
    return op


total = {}
for b in order:
    ins = blocks[b]
    for op in ins:
        total[kind(op)] = total.get(kind(op), 0) + 1
    if len(ins) < min_n and b not in heads:
        continue
    kinds = {}
    for op in ins:
        kinds[kind(op)] = kinds.get(kind(op), 0) + 1
    mark = f"  <- loop head (closed by {', '.join(heads[b])})" if b in heads else ""
    print(f"{b}: {len(ins)} insts {dict(sorted(kinds.items()))}{mark}")
print("kernel total:", dict(sorted(total.items())), sum(total.values()))
for b in dump:
    print(f"\n{b}:")
    for t in text[b]:
        print("   ", t)
