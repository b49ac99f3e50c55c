"""Store-data hazard audit of gfx950 kernel assembly ("The sc1
store failure and its cause").

A vector-memory store of more than 64 bits of data (`*_store_dwordx3`,
`*_store_dwordx4`, and their `_b96` / `_b128` spellings) reads its data
VGPRs after it issues. A VALU instruction that writes one of those registers
within the next 2 wait states on gfx950 (1 on older gfx9; LLVM's
GCNHazardRecognizer, VALU wait states for a VMEM store's data: 2 with GFX940
instructions) can replace the value before the store has read it, so the
store writes whatever the VALU put there. hipcc pads this hazard for the
stores it emits itself; it does not look inside an inline-asm statement
(cdna_hip_programming.md §5.7 item 1: an asm `..._store_dwordx4` must end
with `s_nop 1` in its own string).

Round 3 met it: a build whose bs 32 column-stream epilogue stored C with an
inline-asm `global_store_dwordx4 ... sc1` (write-through) returned 4.8e-42
(the bit pattern of a small integer: the next row's address arithmetic) for
0.8 % of C (profiles/r03_sc1_store_tests.log). tools/history/sc1_store_repro.py
rebuilds that form and this audit names the instruction that overwrote the
data registers.

check(text) walks every function's control-flow graph from each such store,
counting wait states (1 per instruction, N + 1 per `s_nop N`), and reports
every VALU write (mnemonic `v_*`, destination = first operand) of a data
register reached with fewer than WAIT_STATES states elapsed.

Usage: python tools/isa_store_hazard.py <kernel.s> ...
"""
from __future__ import annotations

import re
import sys

import isa_vmcnt as iv

WAIT_STATES = 2  # gfx950 (GFX940 family): VALU write of a VMEM store's data VGPRs
_WIDE_STORE = re.compile(r"^(global|buffer|flat|scratch)_store_(dwordx3|dwordx4|b96|b128)$")
_REG = re.compile(r"\b([va])(?:\[(\d+):(\d+)\]|(\d+)(?!\w))")


def regs(op: str) -> set[tuple[str, int]]:
    """('v' | 'a', index) of every VGPR / AGPR named in one operand."""
    out = set()
    for m in _REG.finditer(op):
        kind = m.group(1)
        if m.group(4) is not None:
            out.add((kind, int(m.group(4))))
        else:
            out |= {(kind, i) for i in range(int(m.group(2)), int(m.group(3)) + 1)}
    return out


def _operands(ops: str) -> list[str]:
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


def store_data(mn: str, ops: str) -> set[tuple[str, int]]:
    """Data registers of a wide store (buffer_*: operand 0; others: operand 1)."""
    o = _operands(ops)
    i = 0 if mn.startswith("buffer_") else 1
    return regs(o[i]) if len(o) > i else set()


def _states(mn: str, ops: str) -> int:
    if mn == "s_nop":
        try:
            return int(ops.split()[0], 0) + 1
        except (ValueError, IndexError):
            return 1
    return 1


def _valu_dest(mn: str, ops: str) -> set[tuple[str, int]]:
    if not mn.startswith("v_") or mn.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
        return set()
    o = _operands(ops)
    return regs(o[0]) if o else set()


def check_function(fname: str, body: list[tuple[int, str]]) -> list[str]:
    blocks = iv.build_cfg(body)
    found = []
    for bi, b in enumerate(blocks):
        for ii, (no, mn, ops) in enumerate(b.insts):
            if not _WIDE_STORE.match(mn):
                continue
            data = store_data(mn, ops)
            in_asm = no in b.asm_lines
            # (block, index of the next instruction, wait states elapsed)
            work = [(bi, ii + 1, 0)]
            seen = set()
            while work:
                cb, ci, st = work.pop()
                if (cb, ci, st) in seen or st >= WAIT_STATES:
                    continue
                seen.add((cb, ci, st))
                blk = blocks[cb]
                if ci >= len(blk.insts):
                    for s in blk.succ:
                        work.append((s, 0, st))
                    continue
                no2, mn2, ops2 = blk.insts[ci]
                hit = _valu_dest(mn2, ops2) & data
                if hit:
                    found.append(f"{fname}: line {no} {mn} {ops} ({'inline asm' if in_asm else 'compiler'})"
                                 f" -> line {no2} {mn2} {ops2} writes {sorted(hit)} after {st} wait"
                                 f" state(s), {WAIT_STATES} needed")
                    continue
                work.append((cb, ci + 1, st + _states(mn2, ops2)))
    return found


def check(text: str) -> dict[str, list[str]]:
    """function -> hazards found (empty list: clean) for every function that
    issues a wide store."""
    res = {}
    for fname, body in iv.split_functions(text).items():
        if any(_WIDE_STORE.match(ln.strip().split(None, 1)[0]) for _, ln in body
               if ln.strip() and not ln.strip().startswith((";", "."))):
            res[fname] = check_function(fname, body)
    return res


def main(argv: list[str]) -> int:
    bad = 0
    for path in argv:
        with open(path) as f:
            res = check(f.read())
        for fn, hz in res.items():
            for h in hz:
                print(h)
            bad += len(hz)
        print(f"{path}: {len(res)} functions with wide stores, {bad} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
