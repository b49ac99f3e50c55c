"""The number tables of README.md and INTEGRATION.md are generated
(tools/gen_tables.py) from one closing pass under profiles/: every marked block
must equal what the script makes of the pass it names, so no number in them is
edited by hand."""
from __future__ import annotations

import importlib.util
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen():
    spec = importlib.util.spec_from_file_location("gen_tables", os.path.join(ROOT, "tools", "gen_tables.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _block(path: str, name: str) -> str:
    with open(os.path.join(ROOT, path)) as f:
        s = f.read()
    m = re.search(rf"<!-- numbers:{name}:begin -->\n(.*?)\n<!-- numbers:{name}:end -->", s, re.S)
    assert m, f"{path}: no numbers:{name} block"
    return m.group(1)


def test_number_blocks_are_generated():
    g = _gen()
    text = _block("README.md", "headline")
    src = re.search(r"From `([^`]+)/bench\.log`", text).group(1)
    head, lines = g.load(os.path.join(ROOT, src))
    assert text == g.headline_table(head, src)
    assert _block("README.md", "workloads") == g.workloads_table(lines, src)
    assert _block("INTEGRATION.md", "entries") == g.entries_table(head, lines, src)
    assert _block("README.md", "sweep") == g.sweep_table(src)


def test_bench_reads_the_same_pass():
    """bench.py's counter-byte records come from the pass the tables quote."""
    text = _block("README.md", "headline")
    src = re.search(r"From `([^`]+)/bench\.log`", text).group(1)
    with open(os.path.join(ROOT, "bench.py")) as f:
        bench = f.read()
    parts = src.split("/")
    for name in ("bsr_bytes.jsonl", "csr_bytes.jsonl"):
        assert f'os.path.join(ROOT, {", ".join(repr(p).replace(chr(39), chr(34)) for p in parts)}, "{name}")' in bench
