"""--write-details (orgscorer.py:766-812, 931-937): the per-iteration gene scores and
gene spans of every clade on an evaluated contig.

Upstream raises on Python 3 (print() into a binary GzipFile), so the fixtures come from
the reference's own write_details() with that one file opened in text mode
(tests/golden/make_details.py); row order within a contig and iteration is clade-name
order (upstream: set order, PYTHONHASHSEED)."""
import gzip
import os

import pytest

import golden_cases as gc
import oracle_bridge as ob
from oracle import orgscorer_oracle as orc

DETAILS = gc.details_names()


def _oracle_text(paths, flags):
    from waafle_amd import cli
    rows = []
    params = orc.Params(**cli.param_dict(cli.parse_flags(flags)))
    orc.run(*paths, params, details=rows)
    head = "CONTIG_NAME\tITERATION\tCLADE\tGENE_SCORES\tGENE_SPANS"
    return "\n".join([head] + ["\t".join(r) for r in rows]) + "\n"


@pytest.mark.parametrize("name", DETAILS)
def test_oracle_matches_reference_details(name, tmp_path):
    fx = gc.load(name)
    paths = gc.materialize(fx, tmp_path)
    assert _oracle_text(paths, fx["flags"]) == fx["details"]


def test_oracle_all_zero_sites_raise(tmp_path):
    fx = gc.load("details_demo_homology_default")
    paths = gc.materialize(fx, tmp_path)
    with pytest.raises(orc.OracleError, match="IndexError"):
        _oracle_text(paths, ["--min-overlap", "0"])


@pytest.mark.gpu
@pytest.mark.parametrize("name", DETAILS)
def test_gpu_details_match_reference(name, tmp_path):
    from waafle_amd import orgscorer
    fx = gc.load(name)
    paths = gc.materialize(fx, tmp_path)
    out = tmp_path / "out"
    out.mkdir()
    orgscorer.main(paths + ["--outdir", str(out), "--basename", "case", "--quiet",
                            "--write-details"] + fx["flags"])
    with gzip.open(os.path.join(str(out), "case.details.tsv.gz"), "rt") as fh:
        assert fh.read() == fx["details"]


@pytest.mark.gpu
def test_gpu_details_all_zero_sites_refused(tmp_path):
    from waafle_amd import orgscorer
    fx = gc.load("details_demo_homology_default")
    paths = gc.materialize(fx, tmp_path)
    with pytest.raises(SystemExit):
        orgscorer.main(paths + ["--outdir", str(tmp_path), "--quiet", "--write-details",
                                "--min-overlap", "0"])


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [[], ["--jump-taxonomy", "1"], ["--weak-loci", "assign-unknown"]])
def test_gpu_details_match_oracle_synthetic(flags, tmp_path):
    """cfg2-shaped synthetic contigs (200 clades): the HIP records against the oracle."""
    from waafle_amd import orgscorer, synth
    sub = str(tmp_path / "in")
    synth.write_text(synth.generate(n=300, genes=8, clades=200, seed=2), sub, "synth")
    paths = [os.path.join(sub, "synth" + e) for e in (".fna", ".blastout", ".gff", ".taxonomy.tsv")]
    out = tmp_path / "out"
    out.mkdir()
    orgscorer.main(paths + ["--outdir", str(out), "--basename", "case", "--quiet",
                            "--write-details"] + flags)
    with gzip.open(os.path.join(str(out), "case.details.tsv.gz"), "rt") as fh:
        got = fh.read()
    want = _oracle_text(paths, flags)
    assert got.count("\n") > 300
    assert got == want
