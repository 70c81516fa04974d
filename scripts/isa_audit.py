#!/usr/bin/env python3
"""ISA audit of one kernel's loops (dev tool, no GPU): per basic block of each loop,
the VALU / SALU / LDS / VMEM instruction counts, and a class breakdown of the VALU
ops, weighted by the measured issue costs of profiles/r01/ubench_encoding_costs.log.

usage: isa_audit.py FILE.s KERNEL_SUBSTRING [--blocks]
"""
import re
import sys
from collections import Counter, OrderedDict

# cycles per wave64 instruction per SIMD
COST = {"f32": 2.4, "int": 2.4, "cvt": 4.0, "mul_int": 4.0, "mad64": 4.6, "cmp": 6.0, "cnd": 4.0, "bfe": 4.0,
        "f64": 4.0, "pk": 8.0, "other": 2.4, "dpp": 2.4}


def vclass(op):
    if op.startswith("v_pk_"):
        return "pk"
    if "f64" in op:
        return "f64"
    if op.startswith(("v_mul_f32", "v_fma_f32", "v_fmac_f32", "v_fmamk_f32", "v_fmaak_f32", "v_add_f32", "v_sub_f32")):
        return "f32"
    if op.startswith("v_cvt"):
        return "cvt"
    if op.startswith(("v_mul_hi", "v_mul_lo", "v_mul_u32", "v_mul_i32")):
        return "mul_int"
    if op.startswith("v_mad_u64") or op.startswith("v_mad_i64") or op.startswith("v_lshl_add_u64"):
        return "mad64"
    if op.startswith("v_cmp"):
        return "cmp"
    if op.startswith("v_cndmask"):
        return "cnd"
    if op.startswith(("v_bfe", "v_bfi", "v_lshl_add", "v_add_lshl", "v_lshl_or", "v_and_or", "v_or3", "v_perm",
                      "v_bitop3", "v_max3", "v_min3", "v_add3")):
        return "bfe"
    if op.startswith(("v_mov", "v_readfirstlane", "v_writelane", "v_readlane")):
        return "other"
    return "int"


def main():
    path, kern = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and kern in l.split(":")[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    labels = {}
    for i in range(start + 1, end + 1):
        l = lines[i].split(";")[0].rstrip()
        m = re.match(r"^(\.LBB\w+):", lines[i])
        if m:
            cur = m.group(1)
            blocks[cur] = []
            labels[cur] = i
            continue
        m = re.match(r"^; %bb\.(\d+):", lines[i])
        if m:
            cur = "%bb." + m.group(1)
            blocks[cur] = []
            labels[cur] = i
            continue
        s = l.strip()
        if not s or s.startswith("."):
            continue
        blocks[cur].append((i, s))
    names = list(blocks)
    pos = {n: k for k, n in enumerate(names)}
    # back edges: a branch in block b to a label at or before b
    loops = []
    for n in names:
        for _, ins in blocks[n]:
            m = re.match(r"s_(c?branch\w*)\s+(\.LBB\w+)", ins)
            if m and m.group(2) in pos and pos[m.group(2)] <= pos[n]:
                loops.append((m.group(2), n))
    for head, tail in loops:
        body = names[pos[head]:pos[tail] + 1]
        tot = Counter()
        print(f"== loop {head} .. {tail}: {len(body)} blocks")
        for b in body:
            c = Counter()
            for _, ins in blocks[b]:
                op = ins.split()[0]
                if op.startswith("v_"):
                    c["VALU"] += 1
                    c["v:" + vclass(op)] += 1
                elif op.startswith("ds_"):
                    c["LDS"] += 1
                elif op.startswith(("global_", "buffer_", "flat_")):
                    c["VMEM"] += 1
                elif op.startswith("s_waitcnt") or op.startswith("s_nop"):
                    c["wait"] += 1
                elif op.startswith("s_"):
                    c["SALU"] += 1
            tot += c
            if "--blocks" in sys.argv:
                print(f"  {b:12s} VALU {c['VALU']:4d} LDS {c['LDS']:3d} VMEM {c['VMEM']:2d} SALU {c['SALU']:3d}  " +
                      " ".join(f"{k[2:]}={v}" for k, v in sorted(c.items()) if k.startswith("v:")))
        cyc = sum(COST[k[2:]] * v for k, v in tot.items() if k.startswith("v:"))
        print(f"  total VALU {tot['VALU']} LDS {tot['LDS']} VMEM {tot['VMEM']} SALU {tot['SALU']}  issue cycles ~{cyc:.0f}")
        print("  classes: " + " ".join(f"{k[2:]}={v}" for k, v in sorted(tot.items()) if k.startswith("v:")))


if __name__ == "__main__":
    main()


def opcodes(path, kern, blocks):
    """Opcode histogram (VALU only) over the named basic blocks of a kernel."""
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and kern in l.split(":")[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    cur, hist = None, Counter()
    for i in range(start + 1, end):
        m = re.match(r"^(\.LBB\w+):", lines[i]) or re.match(r"^; (%bb\.\d+):", lines[i])
        if m:
            cur = m.group(1)
            continue
        s = lines[i].split(";")[0].strip()
        if cur in blocks and s.startswith("v_"):
            hist[s.split()[0]] += 1
    return hist
