"""Counted-vmcnt audit of gfx950 kernel assembly ("counted waits").

The LDS-staged BSR kernels wait for their LDS-DMA copies with a counted
`s_waitcnt vmcnt(N)` (N > 0: the N youngest vector-memory operations may stay
in flight) followed by `s_barrier`. The bs 32 CM4 kernel did that with one
VGPR load (the next A block) younger than the B-panel copies and lost B rows
on the GPU; with every vector-memory operation of the window an LDS-DMA copy
the same kind of wait never failed. Its cause: hipcc deleted
the A loads of the two tail steps of a block row (nothing reads their
values), so in the second tail step the one operation the wait left in flight
was a B copy of the row's last block. A counted wait is only as right as the
instruction stream it counts, so this module checks the stream the compiler
emitted (check_kernel: what a stage hand-off wait keeps in flight and what it
retires; loop_drains: vmcnt(0) waits inside a copy loop that drain the
prefetch). tools/history/vmcnt_order.hip measured the ordering rule itself on the
GPU: a younger VGPR load never retired ahead of an older LDS-DMA copy, nor the
reverse (profiles/r02_vmcnt_order.jsonl).

The checks run per kernel as a forward
dataflow over the control-flow graph. The state at a point is the sequence
(youngest first) of the classes of vector-memory operations that may be in
flight there; at a join the sequences are merged position by position (union
of classes, longer length), which over-approximates every path. `s_waitcnt
vmcnt(N)` truncates the state to its first N positions after the check.

Classes: "dma" (global_load_lds_*, buffer_load_* ... lds), "load" (other
global/buffer/scratch loads, returning atomics), "store" (stores, non-returning
atomics), "flat" (flat_*).

Usage: python tools/isa_vmcnt.py <kernel.s> [name-fragment ...]
"""
from __future__ import annotations

import re
import sys
from dataclasses import dataclass, field

_FUNC_START = re.compile(r"^(_Z\S+|[A-Za-z_][\w.$]*):\s*(;.*)?$")
_LABEL = re.compile(r"^(\.LBB\d+_\d+):")
_NUMLABEL = re.compile(r"^(\d+):\s*$")
_WAIT = re.compile(r"\bvmcnt\((\d+)\)")
MAX_DEPTH = 64


def classify(mn: str, ops: str) -> str | None:
    """Vector-memory class of one instruction, or None."""
    if mn.startswith("flat_"):
        return "flat"
    if mn.startswith("global_load_lds_") or (mn.startswith("buffer_load_") and re.search(r"\blds\b", ops)):
        return "dma"
    if mn.startswith(("global_load_", "buffer_load_", "scratch_load_")):
        return "load"
    if mn.startswith(("global_store_", "buffer_store_", "scratch_store_")):
        return "store"
    if mn.startswith(("global_atomic_", "buffer_atomic_")):
        return "load" if re.search(r"\b(glc|sc0)\b", ops) else "store"
    return None


@dataclass
class Block:
    label: str
    insts: list = field(default_factory=list)  # (line_no, mnemonic, operands)
    succ: list = field(default_factory=list)
    in_loop: bool = False  # the compiler's loop annotation ("in Loop" / "Loop Header")
    header: str = ""       # innermost loop header ("BB12_34") of an in-loop block
    asm_lines: set = field(default_factory=set)  # line numbers inside inline asm


def split_functions(text: str) -> dict[str, list[tuple[int, str]]]:
    """name -> [(line_no, line)] for every function body in the .s file."""
    funcs: dict[str, list[tuple[int, str]]] = {}
    cur = None
    for no, line in enumerate(text.splitlines(), 1):
        if cur is None:
            m = _FUNC_START.match(line)
            if m and not line.startswith(".") and "@function" not in line:
                cur = m.group(1)
                funcs[cur] = []
            continue
        if line.startswith(".Lfunc_end"):
            cur = None
            continue
        funcs[cur].append((no, line))
    return funcs


def build_cfg(body: list[tuple[int, str]]) -> list[Block]:
    """Basic blocks and successors. Numeric local labels of inline asm ("20:",
    targets "20f" / "20b", as in the column-stream kernel's wait ladder) become
    blocks named "20@<n>" and resolve to the next / previous definition."""
    blocks = [Block("<entry>")]
    in_asm = False
    for no, raw in body:
        if "#ASMSTART" in raw:
            in_asm = True
        elif "#ASMEND" in raw:
            in_asm = False
        if re.match(r"^; %bb\.\d+:", raw):  # fall-through block without a label
            blocks.append(Block(raw.split(":")[0][2:]))
        num = _NUMLABEL.match(raw)
        if num:
            blocks.append(Block(f"{num.group(1)}@{len(blocks)}"))
            continue
        m = _LABEL.match(raw)
        if m:
            blocks.append(Block(m.group(1)))
        if "in Loop:" in raw or "Loop Header" in raw:
            blocks[-1].in_loop = True
            h = re.search(r"Header=(BB\d+_\d+)", raw)
            blocks[-1].header = h.group(1) if h else blocks[-1].label.lstrip(".L")
        if m:
            continue
        line = raw.split(";")[0].rstrip()
        if not line.strip():
            continue
        s = line.strip()
        if s.startswith(".") or line[0] not in " \t":
            continue
        parts = s.split(None, 1)
        blocks[-1].insts.append((no, parts[0], parts[1] if len(parts) > 1 else ""))
        if in_asm:
            blocks[-1].asm_lines.add(no)
    index = {b.label: i for i, b in enumerate(blocks)}

    def target(i: int, op: str) -> int:
        t = op.strip().split()[0]
        lm = re.fullmatch(r"(\d+)([fb])", t)
        if not lm:
            return index[t]
        cands = [k for k, b in enumerate(blocks) if b.label.split("@")[0] == lm.group(1)
                 and "@" in b.label]
        return min(k for k in cands if k > i) if lm.group(2) == "f" else max(k for k in cands if k <= i)

    for i, b in enumerate(blocks):
        last = b.insts[-1] if b.insts else None
        fall = True
        # terminators may sit before a trailing non-branch (e.g. s_nop); scan all
        for _, mn, ops in b.insts:
            if mn == "s_branch":
                b.succ.append(target(i, ops))
                fall = False
            elif mn.startswith("s_cbranch_"):
                b.succ.append(target(i, ops))
            elif mn in ("s_endpgm", "s_setpc_b64"):
                fall = False
        del last
        if fall and i + 1 < len(blocks):
            b.succ.append(i + 1)
    return blocks


def _merge(a: tuple, b: tuple) -> tuple:
    """Position-wise union of two in-flight sequences (youngest first); a
    position absent on one path holds the marker "none" (depth differs)."""
    n = max(len(a), len(b))
    none = frozenset(["none"])
    return tuple((a[i] if i < len(a) else none) | (b[i] if i < len(b) else none) for i in range(n))


def _handoff(block: Block, idx: int) -> bool:
    """A wait that hands a stage over: an s_barrier follows it in the same
    block before any other vector-memory instruction."""
    for _, mn, ops in block.insts[idx + 1:]:
        if mn == "s_barrier":
            return True
        if classify(mn, ops) is not None or mn == "s_waitcnt":
            return False
    return False


def _transfer(block: Block, state: tuple, record: list | None, fname: str):
    for i, (no, mn, ops) in enumerate(block.insts):
        if mn == "s_waitcnt":
            m = _WAIT.search(ops)
            if m is None:
                if re.fullmatch(r"\s*0\s*", ops):
                    state = ()
                continue
            n = int(m.group(1))
            if record is not None and n > 0:
                record.append({"kernel": fname, "line": no, "n": n, "handoff": _handoff(block, i),
                               "window": [sorted(x) for x in state[:n + 1]],
                               "depth": len(state)})
            state = state[:n]
            continue
        c = classify(mn, ops)
        if c is not None:
            state = ((frozenset([c]),) + state)[:MAX_DEPTH]
    return state


def counted_waits(fname: str, body: list[tuple[int, str]]) -> list[dict]:
    """Every counted (N > 0) vmcnt wait of one function with the in-flight
    window it sees: positions 0..N-1 stay in flight, position N is the
    youngest operation it retires (merged over every path)."""
    blocks = build_cfg(body)
    ins: list = [None] * len(blocks)
    ins[0] = ()
    work = [0]
    while work:
        i = work.pop()
        out = _transfer(blocks[i], ins[i], None, fname)
        for s in blocks[i].succ:
            new = out if ins[s] is None else _merge(ins[s], out)
            if new != ins[s]:
                ins[s] = new
                work.append(s)
    rec: list[dict] = []
    for i, b in enumerate(blocks):
        if ins[i] is not None:
            _transfer(b, ins[i], rec, fname)
    return sorted(rec, key=lambda r: r["line"])


def issues_dma(body: list[tuple[int, str]]) -> bool:
    for _, line in body:
        t = line.strip().split(None, 1)
        if t and classify(t[0], t[1] if len(t) > 1 else "") == "dma":
            return True
    return False


def check_kernel(fname: str, body: list[tuple[int, str]], keep: str = "dma") -> list[str]:
    """The stage hand-off rule for one LDS-DMA kernel, at every counted wait
    vmcnt(N) followed by s_barrier (merged over every path; "none" marks a
    position that is empty on some path, e.g. after a cursor refill drained
    everything, which only makes the wait stronger):

    keep == "load" (bs 32 CM4: A through VGPRs): the N operations left in
        flight are exactly the A prefetch loads on every path, and the
        youngest operation retired is an LDS-DMA copy on every path — so the
        B copies of the stage handed over are all complete.
    keep == "dma" (every other LDS-staged kernel): the N operations left in
        flight and the youngest one retired are LDS-DMA copies (or nothing) on
        every path — no VGPR load, store or flat access sits in the counted
        window, whose count is planned in copies.
    """
    errs = []
    for r in counted_waits(fname, body):
        if not r["handoff"]:
            continue
        w, n = r["window"], r["n"]
        kept = w[:n]
        retired = w[n] if len(w) > n else ["none"]
        if keep == "load":
            if len(kept) < n or any(x != ["load"] for x in kept):
                errs.append(f"line {r['line']}: vmcnt({n}) keeps {kept}, expected exactly {n} x load")
            if retired != ["dma"]:
                errs.append(f"line {r['line']}: vmcnt({n}) retires {retired} youngest, expected an LDS-DMA copy")
        else:
            if any(not set(x) <= {"dma", "none"} for x in kept):
                errs.append(f"line {r['line']}: vmcnt({n}) keeps {kept} in flight, expected LDS-DMA copies only")
            if not set(retired) <= {"dma", "none"}:
                errs.append(f"line {r['line']}: vmcnt({n}) retires {retired} youngest, expected an LDS-DMA copy")
    return errs


def loop_drains(body: list[tuple[int, str]]) -> list[int]:
    """Lines of vmcnt(0) waits inside a copy loop (one that issues LDS-DMA) that are
    neither a stage hand-off (followed by s_barrier) nor the wait right after a
    VGPR load of the same block (a column-cursor refill used at once). Such a
    wait drains the copies of the blocks ahead in the middle of an iteration,
    which is the prefetch the copy ring exists for."""
    out = []
    blocks = build_cfg(body)
    copy_loops = {b.header for b in blocks
                  if b.in_loop and any(classify(mn, ops) == "dma" for _, mn, ops in b.insts)}
    for b in blocks:
        if not b.in_loop or b.header not in copy_loops:
            continue
        last = None
        for i, (no, mn, ops) in enumerate(b.insts):
            c = classify(mn, ops)
            if c is not None:
                last = c
            elif mn == "s_waitcnt" and (m := _WAIT.search(ops)) and int(m.group(1)) == 0:
                # hand-placed waits in inline asm (the column-stream ladder's
                # exact vmcnt(0) leaf) are not compiler drains
                if last != "load" and not _handoff(b, i) and no not in b.asm_lines:
                    out.append(no)
                last = None
    return out


def audit(text: str, fragments: list[str] | None = None, keep_load: tuple = ("bsr32_f32_cm4_kernel",)):
    """-> {kernel: [errors]} over every LDS-DMA kernel whose name matches."""
    out = {}
    for name, body in split_functions(text).items():
        if fragments and not any(f in name for f in fragments):
            continue
        if not issues_dma(body):
            continue
        keep = "load" if any(k in name for k in keep_load) else "dma"
        out[name] = check_kernel(name, body, keep)
    return out


def _vregs(ops: str) -> set:
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", ops):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def inflight_violations(body: list[tuple[int, str]]) -> list[tuple]:
    """Compiler-generated instructions that touch a register an inline-asm load
    still has in flight. An asm load that does not wait leaves hipcc believing
    its registers hold data at once; they are safe only if nothing but inline asm
    touches them until the consuming asm (which waits, then copies them out with
    v_mov). A forward dataflow over the control-flow graph (union at joins)
    tracks the registers in flight; a full vmcnt(0) lgkmcnt(0) asm wait clears
    them. -> [(line, mnemonic, operands, registers)] (a copy, a spill, a reuse)."""
    stmt_wait, cur, waits = {}, None, False   # asm line -> its statement waits?
    lines_of, drains = [], set()
    for no, line in body:
        if "#ASMSTART" in line:
            cur, waits, lines_of = no, False, []
        elif "#ASMEND" in line:
            for x in lines_of:
                stmt_wait[x] = waits
            cur = None
        elif cur is not None:
            lines_of.append(no)
            waits |= "s_waitcnt" in line
            if "vmcnt(0)" in line and "lgkmcnt(0)" in line:
                drains.add(no)  # a full wait: nothing in flight after it
    blocks = build_cfg(body)
    ins = [None] * len(blocks)
    ins[0] = frozenset()
    errs = []

    def transfer(b, state, report):
        st = set(state)
        for no, mn, ops in b.insts:
            regs = _vregs(ops)
            if no in drains:
                st.clear()
            elif no in stmt_wait:
                if mn.startswith(("global_load_dword", "ds_read")) and not stmt_wait[no]:
                    st |= _vregs(ops.split(",")[0])
                elif mn.startswith("v_mov"):
                    st -= _vregs(ops.partition(",")[2])
            elif regs & st:
                if report:
                    errs.append((no, mn, ops, sorted(regs & st)))
        return frozenset(st)

    work = [0]
    while work:
        bi = work.pop()
        out = transfer(blocks[bi], ins[bi], False)
        for sc in blocks[bi].succ:
            new = out if ins[sc] is None else ins[sc] | out
            if new != ins[sc]:
                ins[sc] = new
                work.append(sc)
    for bi, b in enumerate(blocks):
        if ins[bi] is not None:
            transfer(b, ins[bi], True)
    return errs


def spills(body: list[tuple[int, str]]) -> int:
    return sum(1 for _, line in body if line.strip().startswith("scratch_"))


def inflight_audit(text: str, fragments: list[str]) -> dict:
    """-> {kernel: (spill instructions, in-flight violations)} for the matching kernels:
    run on a TUNING build's assembly before its variants go to the GPU (a variant
    whose allocator spills an asm load's registers in flight reads garbage, and a
    garbage row index is an illegal address)."""
    return {k: (spills(b), inflight_violations(b)) for k, b in split_functions(text).items()
            if any(f in k for f in fragments)}


if __name__ == "__main__" and len(sys.argv) > 2 and sys.argv[1] == "--inflight":
    txt = open(sys.argv[2]).read()
    res = inflight_audit(txt, sys.argv[3:] or ["_cs_kernel", "cs2_kernel", "grp_kernel"])
    bad = 0
    for k, (sp, errs) in res.items():
        print(f"{'FAIL' if errs else 'ok  '} spills {sp:3d}  {k[:100]}")
        for e in errs[:3]:
            print("      ", e)
        bad += bool(errs)
    print(f"{len(res)} kernels, {bad} failing")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    txt = open(sys.argv[1]).read()
    res = audit(txt, sys.argv[2:] or None)
    bad = 0
    for k, errs in res.items():
        waits = [r for r in counted_waits(k, split_functions(txt)[k]) if r["handoff"]]
        print(f"{'FAIL' if errs else 'ok  '} {len(waits):3d} hand-off waits  {k[:100]}")
        for e in errs:
            print("      ", e)
        bad += bool(errs)
    print(f"{len(res)} LDS-DMA kernels, {bad} failing")
    sys.exit(1 if bad else 0)
