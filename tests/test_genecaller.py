"""waafle_genecaller (waafle_genecaller.py:107-233): the CPU oracle against the reference's
shipped golden GFF, the host reader, and (GPU) the HIP path behind wf_genecall against
both."""
import gzip
import os
import random
import shutil

import numpy as np
import pytest

from oracle import genecaller_oracle as gco
from waafle_amd import genecaller as gc

GOLD = os.path.join(os.path.dirname(__file__), "golden", "demo_inputs")


def _unzip(tmp_path, name):
    dest = tmp_path / name
    with gzip.open(os.path.join(GOLD, name + ".gz"), "rb") as fi, open(dest, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    return str(dest)


def _gff_rows(path):
    return [line.rstrip("\n").split("\t") for line in open(path)]


def _synthetic_blastout(path, seed, contigs=40, hits=60):
    """Random overlapping hits (both strands, nested, touching, below --min-scov)."""
    rng = random.Random(seed)
    rows = []
    for c in range(contigs):
        for _ in range(rng.randint(0, hits)):
            a = rng.randint(1, 5000)
            ln = rng.choice([rng.randint(20, 400), rng.randint(300, 1500)])
            b = a + ln - 1
            qs, qe = (a, b) if rng.random() < 0.5 else (b, a)
            slen = ln + rng.randint(0, 60)
            ss = rng.randint(1, slen - ln + 1)
            se = ss + ln - 1
            strand = "plus" if rng.random() < 0.5 else "minus"
            if strand == "minus":
                ss, se = slen - ss + 1, slen - se + 1
            # qseqid sseqid qlen slen length qstart qend sstart send pident positives gaps
            # evalue bitscore sstrand (utils.py:167-183)
            rows.append("c{}\tG{}|s__X\t9000\t{}\t{}\t{}\t{}\t{}\t{}\t{:.3f}\t{}\t0\t0.0\t9\t{}"
                        .format(c, c, slen, ln, qs, qe, ss, se, rng.uniform(70, 100), ln, strand))
    with open(path, "w") as fh:
        fh.write("\n".join(rows) + ("\n" if rows else ""))


def test_oracle_matches_reference_golden_gff(tmp_path):
    blast = _unzip(tmp_path, "demo_contigs.blastout")
    want = _gff_rows(_unzip(tmp_path, "demo_contigs.gff"))
    got = gco.gff_rows(gco.call_genes(blast))
    assert got == want and len(got) == 624


def test_host_reader_groups_like_the_reference(tmp_path):
    blast = _unzip(tmp_path, "demo_contigs.blastout")
    names, off, qs, qe, strand, scov = gc.read_groups(blast)
    ref = [(name, hits) for name, hits in gco.blast_groups(blast)]
    assert names == [n for n, _ in ref]
    assert off[-1] == sum(len(h) for _, h in ref)
    flat = [h for _, hs in ref for h in hs]
    assert qs.tolist() == [h.qstart for h in flat]
    assert strand.tolist() == [1 if h.strand == "-" else 0 for h in flat]
    assert np.array_equal(scov, np.array([h.scov_mod for h in flat]))


def test_oracle_min_overlap_zero_joins_everything(tmp_path):
    path = str(tmp_path / "x.blastout")
    _synthetic_blastout(path, 3, contigs=3, hits=10)
    for contig, genes in gco.call_genes(path, min_overlap=0.0, min_gene_length=0):
        assert len(genes) <= 1


@pytest.mark.gpu
def test_gpu_genecaller_matches_golden_and_oracle(tmp_path):
    blast = _unzip(tmp_path, "demo_contigs.blastout")
    assert gc.call_genes(blast).rows() == _gff_rows(_unzip(tmp_path, "demo_contigs.gff"))
    for seed, kw in [(1, {}), (2, dict(min_overlap=0.5)), (3, dict(min_overlap=0.0)),
                     (4, dict(min_scov=0.0, min_gene_length=0)),
                     (5, dict(min_overlap=1.0, min_gene_length=500))]:
        path = str(tmp_path / "s{}.blastout".format(seed))
        _synthetic_blastout(path, seed)
        want = gco.gff_rows(gco.call_genes(path, **kw))
        got = gc.call_genes(path, **kw).rows()
        assert got == want, (seed, kw)


@pytest.mark.gpu
def test_gpu_genecaller_cli(tmp_path):
    blast = _unzip(tmp_path, "demo_contigs.blastout")
    out = str(tmp_path / "calls.gff")
    gc.main([blast, "--gff", out, "--stranded"])
    assert _gff_rows(out) == _gff_rows(_unzip(tmp_path, "demo_contigs.gff"))
