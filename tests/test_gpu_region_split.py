"""§8f row f4 on the GPU: umiclust.region_split (BGZF on the host threads, record classification and FASTA
emission on the device) against the reference's own outputs on the same inputs (tests/golden/region_split,
made by running region_split.py here with a pysam stand-in, tests/golden/make_golden_region_split.py)."""
import ast
import os

import pytest
from make_golden_region_split import write_inputs
from test_region_split_cpu import cases
from umiclust import region_split as rs

pytestmark = pytest.mark.gpu

SET_LINE = "missing/non-detected regions from reference in initial non-polished read alignments: "


def _norm_log(text):
    """The last line prints a Python set, whose order depends on string hashing: compare it as a set."""
    out = []
    for line in text.splitlines():
        if line.startswith(SET_LINE):
            out.append((SET_LINE, frozenset(ast.literal_eval(line[len(SET_LINE):]) or ())))
        else:
            out.append(line)
    return out


@pytest.mark.parametrize("case", cases(), ids=[c["name"] for c in cases()])
def test_region_split_vs_reference_fixtures(tmp_path, case):
    bam_path, ref_fa, js, out, logs = write_inputs(case, str(tmp_path))
    kw = dict(minimal_region_overlap=case["minimal_region_overlap"], max_softclip_5_end=case["max_softclip_5_end"],
              max_softclip_3_end=case["max_softclip_3_end"])
    if case["error"]:
        exc = KeyError
        with pytest.raises(exc) as e:
            rs.filter_and_split_reads_by_region_cluster(bam_path, js, ref_fa, logs, out, **kw)
        assert f"{exc.__name__}: {e.value}" == case["error"]
    else:
        ret = rs.filter_and_split_reads_by_region_cluster(bam_path, js, ref_fa, logs, out, **kw)
        assert sorted(os.path.relpath(p, str(tmp_path)) for p in ret) == case["result"]
    got = {fn: open(os.path.join(out, fn)).read() for fn in sorted(os.listdir(out))}
    assert got == case["out_files"]
    gl = {fn: _norm_log(open(os.path.join(logs, fn)).read()) for fn in sorted(os.listdir(logs))}
    assert gl == {fn: _norm_log(t) for fn, t in case["log_files"].items()}
