"""Every context option the runtime accepts is documented in the C-ABI header (ofdis.h), with its range.

The option table of `ofdis_context_set_option` (ofdis_runtime.cpp) is the source of truth; VERDICT r02 found
an option (`patch_window`) the header did not mention.  CPU only: the sources are parsed, nothing is run.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def runtime_options():
    src = open(os.path.join(ROOT, "of_dis_amd", "csrc", "ofdis_runtime.cpp")).read()
    table = src[src.index("static const Opt opts[] = {"):]
    table = table[:table.index("};")]
    # the hi field may be an expression ("1 << 30"): evaluated as the C++ constant expression it is
    opts = re.findall(r'\{"(\w+)", &ofdis_context::opt_\w+, (-?\d+), ([^}]+)\}', table)
    assert opts, "option table not found in ofdis_runtime.cpp"
    assert len(opts) == table.count("&ofdis_context::opt_"), "an option entry the pattern does not parse"
    return {k: (int(lo), int(eval(hi, {"__builtins__": {}}))) for k, lo, hi in opts}


def test_every_runtime_option_is_documented():
    hdr = open(os.path.join(ROOT, "include", "ofdis.h")).read()
    missing = [k for k in runtime_options() if not re.search(rf'^ \*\s+"{k}" \(', hdr, re.M)]
    assert not missing, f"options accepted by the runtime but not documented in ofdis.h: {missing}"


def test_documented_ranges_match():
    hdr = open(os.path.join(ROOT, "include", "ofdis.h")).read()
    for k, (lo, hi) in runtime_options().items():
        m = re.search(rf'^ \*\s+"{k}" \(([^)]*)\)', hdr, re.M)
        if not m or k in ("streams", "graph", "chunk"):  # ranges written in words there
            continue
        vals = [int(v) for v in re.findall(r"-?\d+", m.group(1).split(",")[0])]
        if vals:
            assert min(vals) == lo and max(vals) == hi, (k, m.group(1), lo, hi)
