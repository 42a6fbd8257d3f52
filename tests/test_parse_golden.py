"""The consumer counterpart (umiclust.parse_umi_clusters) against golden fixtures produced by running
the reference's parse_umi_clusters.py (tests/golden/make_golden.py)."""
import glob
import json
import os

import pytest
from umiclust.parse_umi_clusters import parse_umi_clusters

FIX = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "parse", "*.json")))


@pytest.mark.parametrize("path", FIX, ids=[os.path.basename(p)[:-5] for p in FIX])
def test_parse_matches_reference(path, tmp_path):
    case = json.load(open(path))
    inp, exp = case["inputs"], case["outputs"]
    d = tmp_path / inp["region"]
    d.mkdir()
    for fn, text in inp["clusters"].items():
        (d / fn).write_text(text)
    (d / "umi_clusters_consensus.fasta").write_text(inp["consout"])
    wo = tmp_path / "regions_wo_clusters.txt"
    kw = dict(inp["args"])
    if inp["region_json"] is not None:
        jp = tmp_path / "region_split_dict.json"
        jp.write_text(json.dumps(inp["region_json"]))
        kw["region_cluster_dict_json"] = str(jp)
    ret = parse_umi_clusters.remote(str(d / "umi_clusters_consensus.fasta"), str(wo), **kw)
    assert (None if ret is None else os.path.relpath(ret, d)) == exp["returned"]
    got = {}
    for root, _dirs, fns in os.walk(d):
        for fn in fns:
            rel = os.path.relpath(os.path.join(root, fn), d)
            if rel in inp["clusters"] or rel == "umi_clusters_consensus.fasta":
                continue
            got[rel] = open(os.path.join(root, fn)).read().replace(str(d), "{DIR}")
    assert got == exp["files"]
    assert (wo.read_text() if wo.exists() else None) == exp["regions_wo"]


def test_parse_refuses_existing_clusters_fa(tmp_path):
    d = tmp_path / "r"
    (d / "clusters_fa").mkdir(parents=True)
    (d / "umi_clusters_consensus.fasta").write_text("")
    with pytest.raises(Exception):
        parse_umi_clusters(str(d / "umi_clusters_consensus.fasta"), str(tmp_path / "wo.txt"))
