"""waafle_junctions + waafle_qc.

CPU: the oracle restatement against the reference-run fixtures (make_junctions.py), the
product's host readers against the oracle, and the QC filter (host code) against the
fixtures.  GPU: the junction table, per-site coverage and gene-pair hits computed by
wf_junctions (through the C-ABI) against the fixtures and against the oracle on larger
seeded sets.  Integer counts and coverage sums are exact; the coverage means and ratio
are float64 computed in the reference's order, compared as the printed text (%.4f) and,
for the oracle cases, bit for bit.
"""
import gzip
import os
import subprocess
import sys

import numpy as np
import pytest

import golden_cases as gc
from oracle import junctions_oracle as jo
from waafle_amd import inputs, junctions, qc, synth, synth_reads

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = gc.junction_names()


def min_sites(fx):
    f = fx["junction_flags"]
    return int(f[f.index("--min-overlap-sites") + 1]) if "--min-overlap-sites" in f else 25


def qc_args(fx):
    f = fx["qc_flags"]
    return int(f[f.index("--min-junction-hits") + 1]) if "--min-junction-hits" in f else 2


def lines(text):
    return text.splitlines()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_junctions(name, tmp_path):
    fx = gc.load_junction(name)
    fna, gff, sam, lgt = gc.materialize_junction(fx, tmp_path)
    assert jo.junction_rows(fna, gff, sam, min_sites(fx)) == lines(fx["junctions"])
    site, gene = jo.detailed_rows(fna, gff, sam, min_sites(fx))
    assert site == lines(fx["site_hits"])
    assert gene == lines(fx["gene_hits"])


@pytest.mark.parametrize("name", NAMES)
def test_oracle_and_product_qc_match_reference(name, tmp_path):
    fx = gc.load_junction(name)
    fna, gff, sam, lgt = gc.materialize_junction(fx, tmp_path)
    jpath = tmp_path / "j.tsv"
    jpath.write_text(fx["junctions"])
    kept, say = jo.qc_filter(lgt, str(jpath), qc_args(fx))
    assert kept == lines(fx["qc_pass"])
    assert say == lines(fx["qc_stderr"])
    out = tmp_path / "qc.out"
    run = subprocess.run([sys.executable, "-m", "waafle_amd.qc", lgt, str(jpath), "--outfile",
                          str(out)] + fx["qc_flags"], capture_output=True, text=True, cwd=REPO)
    assert run.returncode == fx["qc_returncode"] == 0
    assert out.read_text() == fx["qc_pass"]
    assert run.stderr == fx["qc_stderr"]


@pytest.mark.parametrize("name", NAMES[:2])
def test_product_readers_match_oracle(name, tmp_path):
    fx = gc.load_junction(name)
    fna, gff, sam, lgt = gc.materialize_junction(fx, tmp_path)
    lengths = inputs.read_contig_lengths(fna)
    index = {n: i for i, n in enumerate(lengths)}
    pc, m1s, m1e, m2s, m2e, missing = junctions.read_pairs(sam, index)
    want = list(jo.read_pairs(sam))
    assert missing == []
    assert len(pc) == len(want)
    names = list(lengths)
    got = [((names[c], a, b), (names[c], x, y)) for c, a, b, x, y in
           zip(pc.tolist(), m1s.tolist(), m1e.tolist(), m2s.tolist(), m2e.tolist())]
    assert got == [((m1[1], m1[2], m1[3]), (m2[1], m2[2], m2[3])) for m1, m2 in want]
    loci = junctions.read_contig_loci(gff)
    oloci = jo.contig_loci(gff)
    oloci.pop(None, None)
    assert {k: [l.code for l in v] for k, v in loci.items()} == \
        {k: [l.code for l in v] for k, v in oloci.items()}


def test_cigar_length_matches_reference_rule():
    for cig in ["100M", "20S80M", "50M2I48M", "45M5D55M", "60M300N40M", "10H90M", "3M1P2M",
                "5M5X", "1M", "0M", "100=", "MN5", "7MN3M"]:
        try:
            want = jo.cigar_length(cig)
        except ValueError:
            with pytest.raises(ValueError):
                junctions.cigar_length(cig)
            continue
        assert junctions.cigar_length(cig) == want, cig


# ---------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_junctions_cli_matches_reference(name, tmp_path):
    fx = gc.load_junction(name)
    fna, gff, sam, lgt = gc.materialize_junction(fx, tmp_path)
    out = tmp_path / "out"
    out.mkdir()
    junctions.main([fna, gff, "--sam", sam, "--outdir", str(out), "--basename", "case",
                    "--write-detailed-output"] + fx["junction_flags"])
    assert (out / "case.junctions.tsv").read_text() == fx["junctions"]
    assert (out / "case.gene_hits.tsv").read_text() == fx["gene_hits"]
    with gzip.open(str(out / "case.site_hits.tsv.gz"), "rt") as fh:
        assert fh.read() == fx["site_hits"]


@pytest.mark.gpu
@pytest.mark.parametrize("kw,reads,sites", [
    (dict(n=2000, genes=9, clades=50, seed=81, decoys=2), dict(pairs_per_kb=8.0, seed=5), 25),
    (dict(n=500, genes=30, clades=40, seed=82, decoys=1, short_frac=0.4),
     dict(pairs_per_kb=20.0, seed=6, insert=(50, 2000)), 1),
])
def test_gpu_junction_values_bitexact_vs_oracle(kw, reads, sites, tmp_path):
    data = synth.generate(**kw)
    fna, _, gff, _ = synth.write_text(data, str(tmp_path), "s")
    sam = synth_reads.write_sam(data, str(tmp_path / "r.sam"), **reads)
    lengths = inputs.read_contig_lengths(fna)
    names = list(lengths)
    pairs = junctions.read_pairs(sam, {n: i for i, n in enumerate(names)})
    table = junctions.JunctionTable(names, [lengths[n] for n in names],
                                    junctions.read_contig_loci(gff))
    res = junctions.score_junctions(table, pairs, sites, coverage=True, locus_hits=True,
                                    pair_sets=True)
    _, coverage, oloci, hits = jo.accumulate(fna, gff, sam, sites)
    want_cov = np.concatenate([coverage[n] for n in names]).astype(np.int64)
    assert np.array_equal(res["coverage"], want_cov)
    for c, n in enumerate(names):
        cov = coverage[n]
        for j in range(int(table.loc_off[c]), int(table.loc_off[c + 1]) - 1):
            L1, L2 = table.loci[j], table.loci[j + 1]
            gap = L2.start - L1.end - 1
            with np.errstate(invalid="ignore"):
                c1 = np.mean(cov[L1.start - 1:L1.end])
                c2 = np.mean(cov[L2.start - 1:L2.end])
                cj = 0.0 if gap <= 0 else np.mean(cov[L1.end - 1:L2.start])
                ratio = cj / (np.mean([c1, c2]) + 1e-6)
            got = (res["coverage_gene1"][j], res["coverage_gene2"][j],
                   res["coverage_junction"][j], res["ratio"][j])
            for g, w in zip(got, (c1, c2, cj, ratio)):
                assert np.float64(g).tobytes() == np.float64(w).tobytes() or \
                    (np.isnan(g) and np.isnan(w)), (n, j)
            assert res["junction_hits"][j] == hits.get(n, {}).get((L1.code, L2.code), 0)
    assert junctions.gene_hit_rows(table, pairs, res) == jo.detailed_rows(fna, gff, sam, sites)[1]
