"""Lint the counted waits of the MFMA kernels in an emitted gfx950 listing (.s).

The MLP kernels issue their LDS-DMA weight pieces from inline asm, which the compiler's
waitcnt pass does not see, and rounds 1-3 also issued the LDS fragment reads from asm with
compile-time `s_waitcnt lgkmcnt(N)` counts (the NERF_ASM_LDS_READS=1 lab form today).  A
count that is right only for one instruction schedule, or an asm result the register
allocator copies before its wait (what this lint found in round 4), is a silent
wrong-output bug, so this checks the listing the library is built from, instruction by
instruction:

  * every register written by a `ds_read*` (lgkmcnt) or a vector-memory load to registers
    (`global_load*` / `buffer_load*` without `lds`, vmcnt) is pending until a wait retires
    it; LDS ops and vector-memory ops each retire in issue order, so `s_waitcnt
    lgkmcnt(N)` / `vmcnt(N)` retires all but the N youngest of their class (vmcnt also
    counts stores and LDS-DMA pieces, in issue order, as the hardware does);
  * any instruction that reads a pending register, or writes one (the late load would
    clobber it), is a violation -- except a later load of the same in-order class, which
    lands after the older one;
  * scalar memory loads also count in lgkmcnt but return out of order: a wait with
    lgkmcnt(N > 0) while one is outstanding retires nothing of the scalar class and is
    reported if a pending scalar register is then read.

Control flow: basic blocks split at labels and branches; the pending state at a block's
entry is the union over its predecessors (fall-through and every branch to its label),
iterated to a fixed point, so loop back-edges (the persistent tile loop) are covered.

Usage: python tools/lint_waits.py build/asm/mlp_f16x3.s [...]   (exit 1 on a violation)
"""
from __future__ import annotations

import re
import sys
from collections import defaultdict

REG_RE = re.compile(r"\b([vas])\[(\d+):(\d+)\]|\b([vas])(\d+)\b")
LABEL_RE = re.compile(r"^(\.?[A-Za-z_$][\w$.]*):")
FUNC_RE = re.compile(r"^(_Z\w+):")

NO_DST = ("ds_write", "ds_store", "global_store", "buffer_store", "s_waitcnt", "s_cbranch", "s_branch",
          "s_barrier", "s_nop", "s_setprio", "s_sleep", "s_endpgm", "s_cmp", "s_bitcmp", "s_sendmsg",
          "s_dcache", "buffer_inv", "buffer_wbl2", "s_sched", "s_setreg", "s_trap", "s_memtime")


def regs(text):
    out = set()
    for m in REG_RE.finditer(text):
        if m.group(1):
            k, a, b = m.group(1), int(m.group(2)), int(m.group(3))
            out.update((k, i) for i in range(a, b + 1))
        else:
            out.add((m.group(4), int(m.group(5))))
    return {r for r in out if r[0] in "va" or r[0] == "s"}


def split_operands(ops):
    parts, depth, cur = [], 0, ""
    for ch in ops:
        if ch == "[":
            depth += 1
        elif ch == "]":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        parts.append(cur.strip())
    return parts


class Insn:
    __slots__ = ("line", "op", "dst", "src", "text")

    def __init__(self, line, op, dst, src, text):
        self.line, self.op, self.dst, self.src, self.text = line, op, dst, src, text


def parse_insn(lineno, raw):
    text = raw.split(";")[0].strip()
    if not text or text.startswith("."):
        return None
    op, _, rest = text.partition(" ")
    rest = rest.strip()
    # modifiers after the operands (offset:, op_sel:, ...) carry no registers but m0 forms
    ops = split_operands(rest)
    if op.startswith(NO_DST) or "_lds_" in op or (op.startswith("buffer_load") and " lds" in text) \
            or op.startswith("global_load_lds"):
        return Insn(lineno, op, set(), set().union(*[regs(o) for o in ops]) if ops else set(), text)
    if not ops:
        return Insn(lineno, op, set(), set(), text)
    dst = regs(ops[0])
    src = set().union(*[regs(o) for o in ops[1:]]) if len(ops) > 1 else set()
    if op.startswith(("v_fma_mixlo", "v_fma_mixhi", "v_cvt_pk_fp8", "v_cvt_pk_bf8", "v_cvt_scalef32_pk_fp8",
                      "v_mac", "v_fmac")) or "_dpp" in op or "_sdwa" in op or " row_" in text:
        src |= dst                       # partial writes, accumulating ops and DPP read the old value
    if op.startswith("v_cmp") or op.startswith("v_cmpx"):
        dst = {r for r in dst if r[0] == "s"}
    return Insn(lineno, op, dst, src, text)


def classify(ins):
    op = ins.op
    if op.startswith("ds_"):
        loads = bool(ins.dst) and not op.startswith(("ds_write", "ds_store"))
        return "lds", ins.dst if loads else set()
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem", ins.dst
    if op.startswith(("global_load_lds", "global_load", "buffer_load", "global_store", "buffer_store",
                      "global_atomic", "buffer_atomic", "scratch_")):
        if "lds" in ins.text.split(";")[0].split() or op.startswith("global_load_lds") or "_lds_" in op:
            return "vmem", set()
        if op.startswith(("global_store", "buffer_store")):
            return "vmem", set()
        return "vmem", ins.dst
    if op.startswith("flat_"):
        return "flat", ins.dst
    return None, set()


def parse_wait(text):
    vm = lg = None
    m = re.search(r"vmcnt\((\d+)\)", text)
    if m:
        vm = int(m.group(1))
    m = re.search(r"lgkmcnt\((\d+)\)", text)
    if m:
        lg = int(m.group(1))
    if re.fullmatch(r"s_waitcnt\s+0", text.strip()):
        vm, lg = 0, 0
    return vm, lg


class State:
    """Outstanding ops per class as tuples (uid, regs); union-merge keeps the longest history."""

    def __init__(self, lds=(), vmem=(), smem=()):
        self.lds, self.vmem, self.smem = list(lds), list(vmem), list(smem)

    def copy(self):
        return State(self.lds, self.vmem, self.smem)

    def key(self):
        return (tuple(u for u, _ in self.lds), tuple(u for u, _ in self.vmem), tuple(u for u, _ in self.smem))

    def pending(self):
        p = {}
        for cls in ("lds", "vmem", "smem"):
            for uid, rs in getattr(self, cls):
                for r in rs:
                    p[r] = (cls, uid)
        return p


def merge(a, b):
    """Conservative join: per class, the union of outstanding ops, ordered by uid (issue order
    approximated by the uid of the op)."""
    out = State()
    for cls in ("lds", "vmem", "smem"):
        seen = {}
        for uid, rs in getattr(a, cls) + getattr(b, cls):
            seen[uid] = rs
        setattr(out, cls, sorted(seen.items()))
    return out


def lint_function(name, lines):
    # blocks
    insns, labels = [], {}
    for lineno, raw in lines:
        m = LABEL_RE.match(raw.strip())
        if m and not raw.startswith("\t"):
            labels[m.group(1)] = len(insns)
            insns.append(("label", m.group(1), lineno))
            continue
        ins = parse_insn(lineno, raw)
        if ins is not None:
            insns.append(("insn", ins, lineno))
    # block boundaries
    starts = {0}
    for i, (kind, x, _) in enumerate(insns):
        if kind == "label":
            starts.add(i)
        elif x.op.startswith(("s_cbranch", "s_branch", "s_endpgm", "s_setpc")):
            starts.add(i + 1)
    starts = sorted(s for s in starts if s < len(insns))
    blocks = []
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else len(insns)
        blocks.append((s, e))
    block_of_start = {s: bi for bi, (s, e) in enumerate(blocks)}
    label_block = {lab: block_of_start[i] for lab, i in labels.items() if i in block_of_start}
    succ = defaultdict(list)
    for bi, (s, e) in enumerate(blocks):
        last = insns[e - 1]
        fall = True
        if last[0] == "insn":
            op = last[1].op
            if op.startswith(("s_cbranch", "s_branch")):
                tgt = last[1].text.split()[-1]
                if tgt in label_block:
                    succ[bi].append(label_block[tgt])
                if op.startswith("s_branch"):
                    fall = False
            if op.startswith(("s_endpgm", "s_setpc")):
                fall = False
        if fall and bi + 1 < len(blocks):
            succ[bi].append(bi + 1)

    uid_of = {}
    entry = {0: State()}
    violations = []
    changed, it = True, 0
    while changed and it < 12:
        changed, it = False, it + 1
        violations = []
        for bi, (s, e) in enumerate(blocks):
            if bi not in entry:
                continue
            st = entry[bi].copy()
            for i in range(s, e):
                kind, ins, lineno = insns[i]
                if kind != "insn":
                    continue
                if ins.op == "s_waitcnt":
                    vm, lg = parse_wait(ins.text)
                    if lg is not None:
                        st.lds = st.lds[len(st.lds) - lg:] if lg < len(st.lds) else st.lds
                        if lg == 0:
                            st.smem = []
                    if vm is not None:
                        st.vmem = st.vmem[len(st.vmem) - vm:] if vm < len(st.vmem) else st.vmem
                    continue
                pend = st.pending()
                cls, dsts = classify(ins)
                bad_src = ins.src & pend.keys()
                # a later load of the same in-order class may reuse a pending destination: the
                # older load lands first (write-after-write in issue order)
                bad_dst = {r for r in ins.dst & pend.keys() if not (cls in ("lds", "vmem") and pend[r][0] == cls)}
                if bad_src or bad_dst:
                    r = sorted(bad_src | bad_dst)[0]
                    cls, uid = pend[r]
                    violations.append((lineno, ins.text, f"{'reads' if r in bad_src else 'overwrites'} "
                                                         f"{r[0]}{r[1]} pending from {cls} op at line {uid}"))
                if cls in ("lds", "smem", "vmem"):
                    uid = uid_of.setdefault(i, lineno)
                    getattr(st, cls).append((uid, frozenset(dsts)))
                elif cls == "flat":
                    violations.append((lineno, ins.text, "flat memory op (counts in both vmcnt and lgkmcnt)"))
            for sb in succ[bi]:
                new = st if sb not in entry else merge(entry[sb], st)
                if sb not in entry or new.key() != entry[sb].key():
                    entry[sb] = new
                    changed = True
    return violations, sum(1 for k, x, _ in insns if k == "insn")


def functions(path):
    cur, lines = None, []
    for lineno, raw in enumerate(open(path), 1):
        m = FUNC_RE.match(raw)
        if m:
            if cur:
                yield cur, lines
            cur, lines = m.group(1), []
            continue
        if cur is not None:
            if raw.startswith("\t.size") or raw.startswith(".Lfunc_end"):
                yield cur, lines
                cur, lines = None, []
                continue
            lines.append((lineno, raw.rstrip("\n")))
    if cur:
        yield cur, lines


def main(paths):
    bad = 0
    for path in paths:
        for name, lines in functions(path):
            v, n = lint_function(name, lines)
            short = name[:90]
            if v:
                bad += len(v)
                print(f"{path}: {short}: {len(v)} wait violation(s) in {n} instructions")
                for lineno, text, why in v[:20]:
                    print(f"  line {lineno}: {text}   <- {why}")
            else:
                print(f"{path}: {short}: waits cover every LDS / vector-memory result ({n} instructions)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
