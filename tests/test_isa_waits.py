"""The counted vmcnt waits of the LDS-staged BSR kernels, checked on the device
assembly the shipped object is assembled from ("Counted waits").

A copy ring hands a stage to the other waves with `s_waitcnt vmcnt(N)` +
`s_barrier`: N counts the vector-memory operations that may stay in flight,
so it is right only for the instruction stream the compiler emitted. The bs 32
CM4 kernel once lost B rows because hipcc deleted two dead A prefetches in the
tail of a block row and the count then covered a B copy; a GPU rerun loop
caught it about one run in four. These tests read the stream instead:

* every stage hand-off wait keeps in flight only what its kernel plans for
  (LDS-DMA copies) and retires an LDS-DMA copy as its youngest operation, on
  every path (round 1's CM4 kernel, whose ring kept exactly one A prefetch
  load, was removed in round 3; the checker still handles that form);
* no copy loop holds a vmcnt(0) that drains the copies of the blocks ahead in
  the middle of an iteration (hipcc put one before every fp16 B-fragment read
  until those reads went through inline asm);
* the checker flags the pre-fix CM4 tail (a synthetic excerpt of its shape).
"""
from __future__ import annotations

import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "spmm-denseblock_amd")
ASM = os.path.join(PKG, "build", "bsr_kernels-hip-amdgcn-amd-amdhsa-gfx950.s")
sys.path.insert(0, os.path.join(ROOT, "tools"))

import isa_vmcnt as iv  # noqa: E402


@pytest.fixture(scope="module")
def bsr_asm() -> str:
    if not os.path.exists(ASM):
        subprocess.run(["make", "-C", PKG, "lib"], check=True, capture_output=True)
    with open(ASM) as f:
        return f.read()


# The LDS-DMA kernels the library ships (bsr_kernels.hip dispatch): every
# instantiation of each family must be audited.
SHIPPED_DMA = {"bsr32_f32_lds_kernel": 6, "bsr32_f32_cs2_kernel": 20, "bsr16_cm_kernel": 8,
               "bsr16_f16_grp_kernel": 6, "bsr32_f32_grp_kernel": 2,
               "bsr16_f16_cs_kernel": 6}


def test_every_stage_handoff_wait(bsr_asm):
    res = iv.audit(bsr_asm)
    for fam, cnt in SHIPPED_DMA.items():
        got = sum(fam in k for k in res)
        assert got == cnt, f"{fam}: {got} LDS-DMA instantiations audited, expected {cnt}"
    bad = {k: v for k, v in res.items() if v}
    assert not bad, "\n".join(f"{k}: {v}" for k, v in bad.items())


def test_no_copy_loop_drains(bsr_asm):
    drains = {}
    for k, body in iv.split_functions(bsr_asm).items():
        if iv.issues_dma(body) and (d := iv.loop_drains(body)):
            drains[k] = d
    assert not drains, drains


_PRE_FIX_SHAPE = """\
_Z10cm4_shapev:
; %bb.0:
\tglobal_load_lds_dwordx4 v[0:1], off
\tglobal_load_lds_dwordx4 v[0:1], off
\tglobal_load_dwordx4 v[2:5], v[6:7], off
.LBB0_1:                                ; =>This Inner Loop Header: Depth=1
\ts_waitcnt vmcnt(1) lgkmcnt(0)
\ts_barrier
\tglobal_load_lds_dwordx4 v[0:1], off
\tglobal_load_lds_dwordx4 v[0:1], off
\tglobal_load_dwordx4 v[2:5], v[6:7], off
\ts_cbranch_scc1 .LBB0_1
; %bb.2:
\ts_waitcnt vmcnt(1) lgkmcnt(0)
\ts_barrier
\tglobal_load_lds_dwordx4 v[0:1], off
\tglobal_load_lds_dwordx4 v[0:1], off
{TAIL_LOAD}; %bb.3:
\ts_waitcnt vmcnt(1) lgkmcnt(0)
\ts_barrier
\ts_waitcnt vmcnt(0)
\ts_endpgm
.Lfunc_end0:
"""


def test_checker_flags_the_pre_fix_tail():
    """The loop steps load A after their B copies; the first tail step's A
    load was deleted, so the second tail step's vmcnt(1) keeps a B copy."""
    broken = _PRE_FIX_SHAPE.replace("{TAIL_LOAD}", "")
    fixed = _PRE_FIX_SHAPE.replace("{TAIL_LOAD}", "\tglobal_load_dwordx4 v[2:5], v[6:7], off\n")
    body = iv.split_functions(broken)["_Z10cm4_shapev"]
    errs = iv.check_kernel("_Z10cm4_shapev", body, keep="load")
    assert errs and "keeps [['dma']]" in errs[0], errs
    body = iv.split_functions(fixed)["_Z10cm4_shapev"]
    assert iv.check_kernel("_Z10cm4_shapev", body, keep="load") == []


def test_checker_flags_a_mid_loop_drain():
    text = """\
_Z5drainv:
.LBB1_1:                                ; =>This Inner Loop Header: Depth=1
\ts_waitcnt vmcnt(2) lgkmcnt(0)
\ts_barrier
\tglobal_load_lds_dwordx4 v[0:1], off
\tglobal_load_lds_dwordx4 v[0:1], off
\ts_waitcnt vmcnt(0)
\tds_read_b64_tr_b16 v[2:3], v4
\ts_cbranch_scc1 .LBB1_1
; %bb.2:
\ts_endpgm
.Lfunc_end1:
"""
    body = iv.split_functions(text)["_Z5drainv"]
    assert len(iv.loop_drains(body)) == 1


@pytest.mark.parametrize("kernel", ["bsr32_f32_cs2_kernel", "bsr16_f16_cs_kernel",
                                    "bsr16_f16_grp_kernel", "bsr32_f32_grp_kernel"])
def test_column_stream_counts_only_its_copies(bsr_asm, kernel):
    """The column streams wait with counts computed at run time from the
    number of vector-memory operations they issued (A copies, B rows or
    item copies, block-column chunks). That is exact only if every such
    operation in a copy loop is one the wave counts — an LDS-DMA copy or an
    inline-asm load — and the compiler adds no waits of its own: no
    compiler-generated VGPR load, store or spill (scratch) in a copy loop,
    and every vmcnt wait there one of the hand-placed ones (inline asm)."""
    funcs = iv.split_functions(bsr_asm)
    cs = [k for k in funcs if kernel in k]
    assert len(cs) >= (2 if "bsr32_f32_grp" in kernel else 4), "column-stream instantiations"
    for k in cs:
        body = funcs[k]
        assert not any(line.strip().startswith("scratch_") for _, line in body), f"{k}: spills"
        blocks = iv.build_cfg(body)
        # the analysed bs 32 form (MSK, 8th template argument) copies nothing into LDS:
        # its loops are the ones with inline-asm loads
        msk = re.search(r"cs2_kernelI(?:L[bi]\d+E){7}Lb1E", k) is not None
        loops = {b.header for b in blocks
                 if b.in_loop and any(iv.classify(mn, ops) == "dma" or
                                      (msk and iv.classify(mn, ops) == "load" and no in b.asm_lines)
                                      for no, mn, ops in b.insts)}
        assert loops, k
        n_dma = 0
        for b in blocks:
            if not (b.in_loop and b.header in loops):
                continue
            for no, mn, ops in b.insts:
                c = iv.classify(mn, ops)
                assert c in (None, "dma") or (c == "load" and no in b.asm_lines), \
                    f"{k} line {no}: {mn} {ops} in a copy loop"
                n_dma += c == "dma"
                if mn == "s_waitcnt" and "vmcnt" in ops:
                    assert no in b.asm_lines, f"{k} line {no}: compiler-placed {mn} {ops}"
        # the grouped streams at W = 8 (bs 16) / W = 4 (bs 32) issue one copy per wave per
        # item: P = 3 per round
        assert msk or n_dma >= (3 if "grp" in kernel else 4), (k, n_dma)


@pytest.mark.parametrize("kernel", ["bsr32_f32_cs2_kernel", "bsr16_f16_cs_kernel",
                                    "bsr16_f16_grp_kernel", "bsr32_f32_grp_kernel"])
def test_column_stream_registers_in_flight_are_asm_only(bsr_asm, kernel):
    """bsr32_f32_cs2_kernel loads B rows, block-column chunks and A columns
    (bsr16_f16_cs_kernel: block-column chunks; bsr16_f16_grp_kernel: row indices
    and A fragments) with inline asm that does not wait, so hipcc believes their
    registers hold data at once. They are safe only if nothing but inline asm
    touches them while the load is in flight: the consume step's asm waits
    (vmcnt ladder, lgkmcnt(0)) and then copies them out with v_mov.
    tools/isa_vmcnt.py's forward dataflow over the control-flow graph (union at
    joins) tracks the registers in flight; any compiler-generated instruction
    that reads or writes one of them (a copy, a spill, a reuse) fails the test,
    and so does any spill at all in these kernels."""
    funcs = iv.split_functions(bsr_asm)
    cs2 = [k for k in funcs if kernel in k]
    assert len(cs2) >= 2, f"{kernel} instantiations"
    for k in cs2:
        errs = iv.inflight_violations(funcs[k])
        assert not errs, f"{k}: compiler touches in-flight registers: {errs[:5]}"
        assert iv.spills(funcs[k]) == 0, f"{k}: spills"


def test_inflight_check_flags_a_spilled_load():
    """The pattern that faulted a TUNING variant on the GPU (W = 4, P = 3 under
    a 4-waves occupancy hint): the allocator spilled an A fragment whose asm
    load was still in flight."""
    body = [(1, "\t;;#ASMSTART"), (2, "\tglobal_load_dwordx2 v[0:1], v77, s[14:15]"),
            (3, "\t;;#ASMEND"), (4, "\tscratch_store_dwordx2 off, v[0:1], off offset:4"),
            (5, "\t;;#ASMSTART"), (6, "\ts_waitcnt vmcnt(0)"), (7, "\tv_mov_b64 v[2:3], v[0:1]"),
            (8, "\t;;#ASMEND"), (9, "\ts_endpgm")]
    errs = iv.inflight_violations(body)
    assert [e[0] for e in errs] == [4], errs
    assert iv.spills(body) == 1


# ---------------------------------------------------------------------------
# Store-data hazard ("The sc1 store failure"): a VMEM store of
# more than 64 bits reads its data VGPRs after it issues; a VALU write of them
# within 2 wait states (gfx950) replaces the data. hipcc pads its own stores,
# not those inside inline asm, so every shipped object is audited.
# ---------------------------------------------------------------------------
import isa_store_hazard as ish  # noqa: E402

_ALL_ASM = [os.path.join(PKG, "build", f"{k}-hip-amdgcn-amd-amdhsa-gfx950.s")
            for k in ("csr_kernels", "bsr_kernels", "convert_kernels", "f64_kernels",
                      "group_kernels")]


def test_no_store_data_hazard_in_shipped_code():
    if not all(os.path.exists(p) for p in _ALL_ASM):
        subprocess.run(["make", "-C", PKG, "lib"], check=True, capture_output=True)
    total = 0
    for p in _ALL_ASM:
        with open(p) as f:
            res = ish.check(f.read())
        total += len(res)
        bad = {k: v for k, v in res.items() if v}
        assert not bad, "\n".join(h for v in bad.values() for h in v)
    assert total >= 40, f"only {total} functions with wide stores audited"


_HAZARD_EXCERPT = """\
_Z6kernelv:
\tv_mov_b32 v8, s0
\ts_nop 0
\t;;#ASMSTART
\tglobal_store_dwordx4 v[8:9], v[0:3], off sc1
\t;;#ASMEND
\t;;#ASMSTART
\tv_accvgpr_read_b32 v2, a33
\t;;#ASMEND
\ts_nop 1
\t;;#ASMSTART
\tglobal_store_dwordx4 v[8:9], v[4:7], off sc1
\ts_nop 1
\t;;#ASMEND
\tv_mov_b32 v5, 0
\tbuffer_store_dwordx4 v[10:13], v8, s[0:3], 0 offen
\ts_cbranch_scc1 .LBB0_2
.LBB0_1:
\ts_nop 3
.LBB0_2:
\tv_add_u32_e32 v12, 1, v12
\ts_endpgm
.Lfunc_end0:
"""


def test_store_hazard_checker_flags_the_pattern():
    """An asm store followed at once by a VALU write of its data registers is
    flagged (both the straight-line case and the branch that skips the pad);
    a store whose string ends in s_nop 1 is clean."""
    res = ish.check(_HAZARD_EXCERPT)
    hz = res["_Z6kernelv"]
    assert len(hz) == 2, hz
    assert "v_accvgpr_read_b32 v2" in hz[0] and "inline asm" in hz[0]
    assert "v_add_u32_e32 v12" in hz[1]


CSR_ASM = os.path.join(PKG, "build", "csr_kernels-hip-amdgcn-amd-amdhsa-gfx950.s")


def _functions(asm: str, pattern: str) -> dict[str, list[str]]:
    """Instruction lines (labels and comments dropped) of every function whose
    mangled name matches `pattern`."""
    out = {}
    for m in re.finditer(r"^(_Z[^:\s]*(?:" + pattern + r")[^:\s]*):[^\n]*$", asm, re.M):
        body = asm[m.end():asm.index(".Lfunc_end", m.end())]
        out[m.group(1)] = [ln.strip() for ln in body.splitlines()
                           if ln.strip() and not ln.strip().startswith((";", "."))
                           and not ln.strip().endswith(":")]
    return out


def test_split_row_handoff_order_in_shipped_csr_code():
    """The split-row hand-off of the CSR kernels (csr_kernels.hip, split rows) is
    relaxed agent-scope atomics ordered by hand, not by the memory model
    (ADVICE round 4): a wave's partial stores, then s_waitcnt vmcnt(0), then
    its ticket add; the last arriver waits for the add's return before it
    loads the others' partials, with sc1 loads. This pins that order in the
    shipped assembly, path-insensitively (linear order within each function):
      * before the first ticket add, a vmcnt(0) with no vector store after it;
      * after every ticket add, a vmcnt(0) before the next vector load;
      * the partials are read with sc1 loads after the first add, and the
        ticket reset is an sc1 store.
    A compiler that moved a partial store past the wait, or a load above the
    add's return, fails here."""
    if not os.path.exists(CSR_ASM):
        subprocess.run(["make", "-C", PKG, "lib"], check=True, capture_output=True)
    with open(CSR_ASM) as f:
        asm = f.read()
    fns = _functions(asm, "csr_mergepath_kernel|csr_group_kernel")
    assert len(fns) >= 6, f"only {len(fns)} CSR kernel instantiations found"
    is_store = re.compile(r"^(global|buffer)_store")
    is_load = re.compile(r"^(global|buffer)_load")
    for name, ins in fns.items():
        atoms = [i for i, x in enumerate(ins) if x.startswith("global_atomic_add")]
        assert atoms, f"{name}: no ticket add"
        a0 = atoms[0]
        waits = [i for i in range(a0) if re.match(r"s_waitcnt vmcnt\(0\)", ins[i])]
        assert waits, f"{name}: no vmcnt(0) before the first ticket add"
        between = [ins[i] for i in range(waits[-1] + 1, a0) if is_store.match(ins[i])]
        assert not between, f"{name}: stores between the wait and the ticket add: {between}"
        for a in atoms:
            for i in range(a + 1, len(ins)):
                if re.match(r"s_waitcnt vmcnt\(0\)", ins[i]):
                    break
                assert not is_load.match(ins[i]), (
                    f"{name}: {ins[i]!r} before the ticket add's return is waited for")
        after = ins[a0:]
        assert any(is_load.match(x) and " sc1" in x for x in after), f"{name}: no sc1 load"
        assert any(is_store.match(x) and " sc1" in x for x in after), f"{name}: no sc1 store"
