"""Instruction mix of one kernel in a hipcc --save-temps device assembly (.s): per basic block and in total, by
class (MFMA, VALU split into conversion / float / integer-address / select / lane ops, SALU, LDS, global memory,
waits, barriers, branches).  Blocks that a later branch jumps back to are loop heads; the blocks from a loop head to
its back-edge are printed as that loop.
Usage: isa_mix.py <file.s> <mangled-name substring> [--blocks]"""
import collections
import re
import sys


def klass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_read", "ds_load")):
        return "lds_read"
    if op.startswith(("ds_write", "ds_store")):
        return "lds_write"
    if op.startswith("ds_"):
        return "lds_other"
    if op.startswith(("global_load", "buffer_load", "flat_load", "scratch_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store", "scratch_store")):
        return "vmem_store"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        if "cvt" in op or "pk_bf16" in op or "perm" in op:
            return "valu_cvt/perm"
        if op.startswith(("v_readfirstlane", "v_readlane", "v_writelane", "v_mov_b32_dpp")) or "dpp" in op:
            return "valu_lane"
        if "cndmask" in op or op.startswith("v_cmp"):
            return "valu_cmp/select"
        if "_f32" in op or "_f64" in op or "_f16" in op or "pk_add" in op or "pk_mul" in op or "pk_fma" in op:
            return "valu_float"
        if op.startswith("v_mov") or op.startswith("v_accvgpr"):
            return "valu_mov"
        return "valu_int/addr"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    text = open(path).read().splitlines()
    start = None
    for i, l in enumerate(text):
        if l.startswith(name) or (re.match(r"^_Z\S*:", l) and name in l):
            start = i
            break
    if start is None:
        sys.exit(f"no function matching {name}")
    fname = text[start].rstrip(":")
    blocks, order, cur = collections.OrderedDict(), [], "entry"
    blocks[cur] = []
    order.append(cur)
    for l in text[start + 1:]:
        if l.startswith(".Lfunc_end") or re.match(r"^_Z\S*:", l):
            break
        s = l.strip()
        if not s or s.startswith((";", ".", "//")):
            m = re.match(r"^(\.LBB\S+):", s)
            if m:
                cur = m.group(1)
                blocks[cur] = []
                order.append(cur)
            continue
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        op = s.split()[0]
        blocks[cur].append((op, s))
    # back edges: a branch in block b to a label at or before b
    pos = {b: k for k, b in enumerate(order)}
    loops = []
    for b in order:
        for op, s in blocks[b]:
            if op.startswith(("s_cbranch", "s_branch")):
                tgt = s.split()[-1]
                if tgt in pos and pos[tgt] <= pos[b]:
                    loops.append((tgt, b))
    print(fname)
    tot = collections.Counter(klass(op) for b in order for op, _ in blocks[b])
    print(f"total {sum(tot.values())} instructions:", dict(tot.most_common()))
    for head, tail in sorted(set(loops), key=lambda x: pos[x[0]]):
        c = collections.Counter(klass(op) for b in order[pos[head]:pos[tail] + 1] for op, _ in blocks[b])
        print(f"loop {head} .. {tail} ({pos[tail] - pos[head] + 1} blocks) {sum(c.values())} instructions:",
              dict(c.most_common()))
    if "--blocks" in sys.argv:
        for b in order:
            c = collections.Counter(klass(op) for op, _ in blocks[b])
            if c:
                print(f"  {b}: {sum(c.values())}", dict(c.most_common()))


if __name__ == "__main__":
    main()
