#!/usr/bin/env python3
"""The number tables of README.md / INTEGRATION.md, generated from one closing pass.

    python tools/gen_tables.py profiles/r06_final            # print the tables
    python tools/gen_tables.py profiles/r06_final --write    # rewrite the marked blocks

Reads the pass's `bench.log` (the default bench line: the headline with its BASELINE config
3 / config 5 / products bs 32 side entries and the CPU baseline) and `workloads.jsonl` (one
bench line per workload), and replaces everything between `<!-- numbers:NAME:begin -->` and
`<!-- numbers:NAME:end -->` in README.md (NAME = headline, workloads, sweep) and INTEGRATION.md
(NAME = entries). No number in those blocks is typed by hand.
"""
from __future__ import annotations

import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# what each workload line is, in the order the table lists them
WORKLOADS = [
    ("products_csr_k256", "CSR, products stand-in (2.45 M rows, 61.9 M nnz), K = 256 (config 4 shape, 1 GPU)"),
    ("products_csr_hot", "CSR with hot-column hints (analysis once), products stand-in, K = 128"),
    ("arxiv_csr", "CSR, arxiv stand-in (169 K rows, 1.17 M nnz), K = 128 (config 2)"),
    ("reddit_bsr32", "BSR bs 32 fp32 drop-in, reddit stand-in, K = 128 (config 3)"),
    ("reddit_bsr32_an", "the same, analysed entry"),
    ("reddit_bsr32_grp", "the same, grouped entry (W = 2)"),
    ("reddit_rcm_bsr32", "BSR bs 32 drop-in after in-repo RCM of scrambled ids, reddit"),
    ("reddit_rcm_bsr32_an", "the same, analysed entry"),
    ("products_bsr32", "BSR bs 32 fp32 drop-in, products stand-in, K = 128 (north_star's BSR target)"),
    ("products_bsr32_an", "the same, analysed entry"),
    ("products_bsr32_grp", "the same, grouped entry (W = 2)"),
    ("products_rcm_bsr32", "BSR bs 32 drop-in after RCM, products"),
    ("products_rcm_bsr32_an", "the same, analysed entry"),
    ("products_bsr16_f16", "BSR bs 16 fp16 drop-in, products stand-in, K = 512 (config 5)"),
    ("products_bsr16_f16_an", "the same, analysed entry"),
    ("products_bsr16_f16_grp", "the same, grouped entry (W by the library)"),
    ("products_rcm_bsr16_f16", "BSR bs 16 fp16 drop-in after RCM, products, K = 512"),
    ("products_rcm_bsr16_f16_grp", "the same, grouped entry"),
    ("reddit_bsr8", "BSR bs 8 fp32 drop-in, reddit stand-in, K = 128"),
    ("reddit_bsr4", "BSR bs 4 fp32 drop-in, reddit"),
    ("reddit_bsr2", "BSR bs 2 fp32 drop-in, reddit"),
    ("reddit_bsr64", "BSR bs 64 fp32 drop-in, reddit"),
    ("reddit_bsr8_rb32", "bs 8 re-blocked to 32 once + analysed bs 32"),
    ("reddit_bsr4_rb32", "bs 4 re-blocked to 32 once + analysed bs 32"),
    ("reddit_bsr2_rb32", "bs 2 re-blocked to 32 once + analysed bs 32"),
    ("reddit_hybrid32", "hybrid dense-block bs 32 + CSR remainder, reddit"),
    ("products_hybrid32", "hybrid dense-block bs 32 + CSR remainder, products"),
]


def _f(x, nd=3):
    return "" if x is None else f"{x:.{nd}f}"


def _wl(rec) -> str:
    return rec["config"]["workload"].split(":")[0]


def load_bytes(pass_dir: str) -> dict:
    """Counter bytes per launch by workload (tools/pmc_bytes.sh records of the same pass):
    the lines were measured before those records existed, so their `traffic` is filled
    from here where it is missing."""
    out = {}
    for name in ("csr_bytes.jsonl", "bsr_bytes.jsonl"):
        path = os.path.join(pass_dir, name)
        if not os.path.exists(path):
            continue
        with open(path) as f:
            for line in f:
                if line.startswith("{"):
                    r = json.loads(line)
                    if r.get("counter_bytes_per_launch"):
                        out[r["workload"]] = r
    return out


def load(pass_dir: str):
    head = None
    with open(os.path.join(pass_dir, "bench.log")) as f:
        for line in f:
            if line.startswith("{"):
                head = json.loads(line)
    lines = {}
    cb = load_bytes(pass_dir)
    path = os.path.join(pass_dir, "workloads.jsonl")
    if os.path.exists(path):
        with open(path) as f:
            for line in f:
                if line.startswith("{"):
                    r = json.loads(line)
                    rf = r.setdefault("roofline", {})
                    if not rf.get("traffic") and _wl(r) in cb:
                        rf["traffic"] = cb[_wl(r)]["counter_bytes_per_launch"]
                    lines[_wl(r)] = r
    if head:
        rf = head["roofline"]
        if not rf.get("traffic") and "products_csr" in cb:
            rf["traffic"] = cb["products_csr"]["counter_bytes_per_launch"]
        for key, wl in (("config3", "reddit_bsr32"), ("config5", "products_bsr16_f16"),
                        ("products_bsr32", "products_bsr32")):
            s = head.get(key)
            if not s:
                continue
            for sub, suf in ((s, ""), (s.get("grouped_entry"), "_grp"), (s.get("analysed_entry"), "_an")):
                rec = cb.get(wl + suf)
                if sub is not None and not sub.get("traffic") and rec:
                    sub["traffic"] = rec["counter_bytes_per_launch"]
                    if sub is s and sub.get("kernel_ms"):
                        sub["traffic_frac"] = rec["counter_bytes_per_launch"] / (sub["kernel_ms"] * 1e-3) / 8e12
    return head, lines


def headline_table(h: dict, src: str) -> str:
    rf = h["roofline"]
    cpu = h.get("cpu_baseline") or {}
    out = [f"From `{src}/bench.log` (the driver's default `python bench.py` line, one MI355X):", "",
           "| Line | ms / step | kernel ms | GFLOP/s | roofline | counter bytes | MFMA executed |",
           "|---|---|---|---|---|---|---|"]
    tr = rf.get("traffic")
    tcell = f"{tr / 1e9:.2f} GB / launch" if tr else ""
    out.append(f"| headline: CSR, products stand-in, K = 128 (`value`) | {h['ms_per_step']:.3f} | "
               f"{rf.get('kernel_ms', 0):.3f} | {h['value']:.0f} | {rf['frac']:.3f} of 8 TB/s "
               f"({rf['achieved'] / 1000:.2f} TB/s algorithmic) | {tcell} | |")
    hot = h.get("hot_column_hints")
    if hot:
        out.append(f"| the same on hot-column hints (analysis {hot.get('analysis_ms_first_call', 0):.2f} ms once) | "
                   f"{hot.get('ms_per_step', 0):.3f} | {_f(hot.get('kernel_ms'))} | "
                   f"{_f(hot.get('value'), 0)} | | | |")
    for key, name in (("config3", "config 3: reddit bs 32 fp32, drop-in"),
                      ("config5", "config 5: products bs 16 fp16 K = 512, drop-in"),
                      ("products_bsr32", "products bs 32 fp32 K = 128, drop-in")):
        s = h.get(key)
        if not s:
            continue
        tb, tf = s.get("traffic"), s.get("traffic_frac") or 0.0
        tcell = f"{tb / 1e9:.2f} GB ({tf:.3f} of 8 TB/s)" if tb else ""
        out.append(f"| {name} | {s['ms_per_step']:.3f} | {s['kernel_ms']:.3f} | {s['value']:.0f} | "
                   f"{s['roofline_frac']:.3f} of 8 TB/s (compulsory bytes) | {tcell} | "
                   f"{_f(s.get('mfma_frac'))} |")
        for e, en in (("grouped_entry", "grouped"), ("analysed_entry", "analysed")):
            g = s.get(e)
            if not g:
                continue
            an = g.get("analysis_ms_repeat")
            acell = "" if an is None else f" (analysis {an:.2f} ms once)"
            fcell = "" if g.get("frac") is None else f"{g['frac']:.3f}"
            gcell = f"{g['traffic'] / 1e9:.2f} GB" if g.get("traffic") else ""
            out.append(f"| ... {en} entry{acell} | {g['ms_per_step']:.3f} | {g['kernel_ms']:.3f} | | "
                       f"{fcell} | {gcell} | {_f(g.get('mfma_frac'))} |")
    if cpu:
        out += ["", f"CPU baseline (`spmm.cc` `csr_spmm` restated, {cpu.get('cores')} threads on the GPU "
                f"box's host, {cpu.get('kind')}): {cpu.get('value')} {cpu.get('unit')} on {cpu.get('sample')}."]
    return "\n".join(out)


def workloads_table(lines: dict, src: str) -> str:
    out = [f"From `{src}/workloads.jsonl` (`bench.py --workload W`, 20 steps after 5 warm-up, one MI355X):",
           "", "| Workload | ms / step | kernel ms | GFLOP/s (2 nnz K / t) | roofline (compulsory bytes) "
           "| counter GB / launch | fp32 or fp16 MFMA executed | analysis ms once | CSR on the same matrix, ms |",
           "|---|---|---|---|---|---|---|---|---|"]
    for key, desc in WORKLOADS:
        r = lines.get(key)
        if not r:
            continue
        rf = r.get("roofline") or {}
        tr = rf.get("traffic")
        tcell = f"{tr / 1e9:.2f}" if tr else ""
        out.append(f"| `{key}`: {desc} | {r['ms_per_step']:.3f} | {_f(rf.get('kernel_ms'))} | "
                   f"{r['value']:.0f} | {_f(rf.get('frac'))} | {tcell} | "
                   f"{_f(rf.get('mfma_frac'))} | {_f(r.get('analysis_ms'), 2)} | "
                   f"{_f(r.get('csr_same_matrix_ms'), 2)} |")
    return "\n".join(out)


def entries_table(h: dict, lines: dict, src: str) -> str:
    """The INTEGRATION.md view: each entry point the reference's calls map to, on its config."""
    rows = []

    def add(entry, wl, r, extra=""):
        if r:
            rows.append(f"| `{entry}` | {wl} | {r['ms_per_step']:.3f} | {extra} |")
    add("spmm_gespmm_csrmm_f32 (gespmm_csrmm<float>)", "products stand-in, K = 128",
        {"ms_per_step": h["ms_per_step"]}, "headline")
    hot = h.get("hot_column_hints")
    if hot:
        add("spmm_csrmm_hot_f32", "products stand-in, K = 128", hot,
            f"after `spmm_csr_hot_analysis` ({hot.get('analysis_ms_first_call', 0):.2f} ms once)")
    for key, wl in (("config3", "reddit bs 32, K = 128"), ("config5", "products bs 16 fp16, K = 512"),
                    ("products_bsr32", "products bs 32, K = 128")):
        s = h.get(key)
        if not s:
            continue
        add("spmm_sbsrmm / rocsparse_bsrmm_template" if key != "config5" else "spmm_bsrmm_ex_f16",
            wl, s)
        g = s.get("grouped_entry")
        if g:
            add("spmm_bsrmm_grouped_f16" if key == "config5" else "spmm_bsrmm_grouped_f32", wl, g,
                f"after the group analysis ({g.get('analysis_ms_repeat', 0):.2f} ms once)")
        a = s.get("analysed_entry")
        if a:
            add("spmm_bsrmm_analysed_f16" if key == "config5" else "spmm_bsrmm_analysed_f32", wl, a,
                "after the column-mask analysis")
    for key, entry, wl in (("reddit_bsr8", "spmm_sbsrmm (bs 8)", "reddit stand-in, K = 128"),
                           ("reddit_bsr2", "spmm_sbsrmm (bs 2)", "reddit stand-in, K = 128"),
                           ("reddit_hybrid32", "spmm_hybrid_csrmm_f32", "reddit stand-in, bs 32, K = 128"),
                           ("products_hybrid32", "spmm_hybrid_csrmm_f32", "products stand-in, bs 32, K = 128")):
        add(entry, wl, lines.get(key))
    out = [f"From `{src}` (one MI355X; the full table is in README.md):", "",
           "| Entry | Input | ms / product | Note |", "|---|---|---|---|"] + rows
    return "\n".join(out)


def sweep_table(src: str) -> str:
    """The reference's own benchmark sweep (benchmark.py:3-31) of the pass, as
    tools/ref_sweep.py --table prints it."""
    import contextlib
    import importlib.util
    import io
    spec = importlib.util.spec_from_file_location("ref_sweep", os.path.join(ROOT, "tools", "ref_sweep.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        mod.table(os.path.join(ROOT, src, "sweep.jsonl"))
    return (f"From `{src}/sweep.jsonl` (`tools/ref_sweep.py`: the reference's own "
            f"`benchmark.py` sweep on 131,072² random matrices, one MI355X):\n\n"
            + buf.getvalue().rstrip("\n"))


def replace_block(path: str, name: str, text: str) -> None:
    with open(path) as f:
        s = f.read()
    pat = re.compile(rf"(<!-- numbers:{name}:begin -->\n).*?(<!-- numbers:{name}:end -->)", re.S)
    if not pat.search(s):
        raise SystemExit(f"{path}: no numbers:{name} block")
    s = pat.sub(lambda m: m.group(1) + text + "\n" + m.group(2), s)
    with open(path, "w") as f:
        f.write(s)


def main() -> None:
    src = sys.argv[1] if len(sys.argv) > 1 else "profiles/r06_final"
    head, lines = load(os.path.join(ROOT, src))
    tables = {"headline": headline_table(head, src), "workloads": workloads_table(lines, src),
              "entries": entries_table(head, lines, src), "sweep": sweep_table(src)}
    if "--write" in sys.argv:
        replace_block(os.path.join(ROOT, "README.md"), "headline", tables["headline"])
        replace_block(os.path.join(ROOT, "README.md"), "workloads", tables["workloads"])
        replace_block(os.path.join(ROOT, "README.md"), "sweep", tables["sweep"])
        replace_block(os.path.join(ROOT, "INTEGRATION.md"), "entries", tables["entries"])
    else:
        for k, v in tables.items():
            print(f"## {k}\n\n{v}\n")


if __name__ == "__main__":
    main()
