#!/usr/bin/env python3
"""Instruction mix of the loops (backward branches) of one kernel in an llvm-objdump -d listing.
    python bench/probe/asm_loops.py listing.s <kernel symbol substring>"""
import re
import sys
from collections import Counter

lines = open(sys.argv[1]).read().split("\n")
key = sys.argv[2]
start = next(i for i, l in enumerate(lines) if key in l and l.endswith(">:"))
base = int(re.match(r"^([0-9a-f]+)", lines[start]).group(1), 16)
ins = []
for l in lines[start + 1:]:
    if re.match(r"^[0-9a-f]+ <.*>:$", l):
        break
    m = re.match(r"\s+(\S+)\s*(.*?)\s*//\s*([0-9A-F]+):", l)
    if m:
        t = re.search(r"\+0x([0-9a-f]+)>", l)
        ins.append((int(m.group(3), 16) - base, m.group(1), m.group(2), int(t.group(1), 16) if t else None))
loops = [(t, a) for a, op, _, t in ins if t is not None and t < a and op.startswith("s_")]
loops = sorted(set(loops), key=lambda x: x[1] - x[0], reverse=True)
print(f"{len(ins)} instructions, {len(loops)} loops")
for t, a in loops[:6]:
    body = [x for x in ins if t <= x[0] <= a]
    c = Counter()
    for _a, op, args, _t in body:
        if op.startswith("v_fma_f64") or op.startswith("v_mul_f64") or op.startswith("v_add_f64") or \
                op.startswith("v_fmac_f64") or op.startswith("v_div") or op.startswith("v_rcp_f64"):
            c["valu f64 arith"] += 1
        elif op.startswith("v_cvt"):
            c["valu cvt"] += 1
        elif op.startswith("v_cndmask"):
            c["valu cndmask"] += 1
        elif op.startswith("v_mov") and "dpp" in args:
            c["valu dpp mov"] += 1
        elif op.startswith("v_mov") or op.startswith("v_accvgpr"):
            c["valu mov"] += 1
        elif op.startswith("v_"):
            c["valu other"] += 1
        elif op.startswith("global_load") or op.startswith("buffer_load"):
            c["vmem load"] += 1
        elif op.startswith("global_store") or op.startswith("buffer_store"):
            c["vmem store"] += 1
        elif op.startswith("s_waitcnt"):
            c["s_waitcnt"] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            c["smem load"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("s_"):
            c["salu/branch"] += 1
        else:
            c[op] += 1
    print(f"loop [{t:#x}, {a:#x}] {len(body)} instructions: " + ", ".join(f"{k} {v}" for k, v in c.most_common()))
