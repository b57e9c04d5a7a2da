"""Native ingest (libwaafle_ingest.so) against the Python reader:
identical HostBatch / taxonomy on every golden input and on synthetic text, the same
warnings, and the Python reader's result or error wherever the native parser hands over."""
import os

import numpy as np
import pytest

import golden_cases as gc
from waafle_amd import cli, ingest, inputs, synth
from waafle_amd.taxonomy import read_edges

ARRAYS = ("contig_lengths", "hit_off", "hit_qlo", "hit_qhi", "hit_taxon", "hit_strand",
          "hit_score", "hit_scov", "hit_sysmask", "loc_off", "loc_start", "loc_end",
          "loc_strand", "hit_row")


def both(paths, mgl, threads=0):
    warn_n, warn_p = [], []
    bn, tn = inputs.load_inputs(*paths, mgl, warn=lambda *a: warn_n.append(a), native=True,
                                threads=threads)
    bp, tp = inputs.load_inputs(*paths, mgl, warn=lambda *a: warn_p.append(a), native=False)
    return (bn, tn, warn_n), (bp, tp, warn_p)


def native_only(paths, mgl, threads=0):
    edges = read_edges(paths[3])
    return ingest.parse(paths[0], paths[1], paths[2], edges, mgl, threads=threads)


def assert_same(a, b):
    bn, tn, wn = a
    bp, tp, wp = b
    assert wn == wp
    assert (bn.hit_group is None) == (bp.hit_group is None)
    if bn.hit_group is not None:
        assert np.array_equal(bn.hit_group, bp.hit_group)
    assert tn.names == tp.names
    assert bn.contig_names == bp.contig_names
    for f in ARRAYS:
        x, y = getattr(bn, f), getattr(bp, f)
        assert x.dtype == y.dtype, f
        assert np.array_equal(x, y), f
    assert bn.loc_codes == bp.loc_codes
    assert bn.systems == bp.systems
    # annotation values: compare the resolved strings (ids are per-reader numbering)
    for h in range(bn.n_hits):
        for s in range(len(bn.systems)):
            i, j = bn.annot_value_ids[h, s], bp.annot_value_ids[h, s]
            assert (i < 0) == (j < 0)
            if i >= 0:
                assert bn.annot_values[s][i] == bp.annot_values[s][j]


@pytest.mark.parametrize("name", gc.case_names())
def test_golden_inputs_native_equals_python(name, tmp_path):
    fx = gc.load(name)
    paths = gc.materialize(fx, tmp_path)
    args = cli.parse_flags(fx["flags"])
    native_only(paths, args.min_gene_length)          # takes the native path (no fallback)
    a, b = both(paths, args.min_gene_length)
    assert_same(a, b)


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_synthetic_text_native_equals_python(tmp_path, threads):
    data = synth.generate(n=300, genes=6, clades=40, seed=11)
    paths = synth.write_text(data, str(tmp_path))
    a, b = both(paths, 200.0, threads=threads)
    assert_same(a, b)
    batch, _ = native_only(paths, 200.0, threads=threads)
    assert batch.n_hits == data.n_hits


def _write(tmp_path, fna, blast, gff, tax="s__A\tg__A\ns__B\tg__A\ng__A\tr__Root\n"):
    paths = []
    for name, text in (("c.fna", fna), ("c.blastout", blast), ("c.gff", gff), ("t.tsv", tax)):
        p = os.path.join(str(tmp_path), name)
        with open(p, "w", newline="") as fh:
            fh.write(text)
        paths.append(p)
    return paths


FNA = ">c1 desc\nACGT\nAC\n>c2\nAAAAAAAAAA\n>c1\nGG\n"
GFF = ("##gff-version 3\nc1\tx\tgene\t1\t300\t.\t+\t0\tid=1\n"
       "c9\tx\tgene\t1\t300\t.\t+\t0\tid=9\nc2\tx\tgene\t400\t100\t1.5\t-\t0\tid=2\n"
       "c2\tx\tgene\t1\t50\t.\t.\t0\tid=3\n")


def _row(q, sid, qs=1, qe=300, ss=1, se=300, slen=300, pid="95.5", strand="plus"):
    return "\t".join(map(str, [q, sid, 1000, slen, abs(qe - qs) + 1, qs, qe, ss, se, pid, 10, 0,
                               "1e-50", "300", strand])) + "\n"


BLAST = (_row("c1", "g1|s__A|SYS=v1|K=k") + _row("c1", "g2|s__B", pid="80") +
         _row("c9", "g3|s__Z|Q=z") + _row("c2", "g4|s__A|SYS=v2|SYS=v3", strand="minus", ss=300, se=1) +
         _row("c2", "g5|s__B|K=k", qs=120, qe=380))


def test_crlf_line_ends_match(tmp_path):
    """Universal newlines: "\r\n" ends a line like "\n" (the demo GFF uses it)."""
    paths = _write(tmp_path, FNA.replace("\n", "\r\n"), BLAST.replace("\n", "\r\n"),
                   GFF.replace("\n", "\r\n"))
    native_only(paths, 100)
    assert_same(*both(paths, 100))


def test_edge_semantics_match(tmp_path):
    """Repeated FASTA header (OrderedDict), comments, unknown contigs (warnings in order),
    dotted scores, odd strands, minus-strand hits, repeated annotation systems."""
    paths = _write(tmp_path, FNA, BLAST, GFF)
    native_only(paths, 100)
    a, b = both(paths, 100)
    assert_same(a, b)
    bn = a[0]
    assert bn.contig_names == ["c1", "c2"] and list(bn.contig_lengths) == [2, 10]
    assert [w[0].strip() for w in a[2]] == ["Unknown contig in <gff> file",
                                            "Unknown contig in <blastout> file"]
    assert bn.systems == ["K", "SYS"]


@pytest.mark.parametrize("blast,gff,why", [
    (BLAST.replace("95.5", " 95.5"), GFF, "space in a float"),
    (BLAST.replace("\t1000\t", "\t+1_000\t", 1), GFF, "underscore int"),
    (BLAST.replace("g1|s__A", '"g1|s__A"'), GFF, "quoted field"),
    (BLAST.replace("\tplus\n", "\tplus\rx\n", 1), GFF, "lone CR"),
    (BLAST, GFF.replace("\t1\t300\t", "\t 1\t300\t", 1), "space in a GFF int"),
])
def test_unusual_spelling_goes_to_python_reader(tmp_path, blast, gff, why):
    paths = _write(tmp_path, FNA, blast, gff)
    with pytest.raises(ingest.Fallback):
        native_only(paths, 100)
    try:
        want = inputs.load_inputs(*paths, 100, warn=None, native=False)
    except (inputs.InputError, ValueError) as exc:
        with pytest.raises(type(exc)):
            inputs.load_inputs(*paths, 100, warn=None, native=True)
        return
    got = inputs.load_inputs(*paths, 100, warn=None, native=True)
    assert got[0].n_hits == want[0].n_hits
    assert np.array_equal(got[0].hit_score, want[0].hit_score)


@pytest.mark.parametrize("blast,gff", [
    (BLAST.replace("\t0\t1e-50", "\t0\t1e-50\textra", 1), GFF),          # 16 columns
    (BLAST.replace("\t1000\t300\t", "\t1000\t0\t", 1), GFF),             # slen 0
    (BLAST.replace("g2|s__B", "g2"), GFF),                               # bad sseqid
    (BLAST.replace("SYS=v1", "SYSv1"), GFF),                             # bad annotation
    (BLAST, GFF + "c1\tx\tgene\t1\t300\t.\t+\t0\tid=1\n"),               # ungrouped GFF
    (BLAST, GFF.replace("\t1.5\t", "\tabc\t")),                          # bad GFF score
    (BLAST, GFF + "\n"),                                                 # blank GFF line
])
def test_malformed_inputs_raise_the_python_error(tmp_path, blast, gff):
    paths = _write(tmp_path, FNA, blast, gff)
    with pytest.raises(ingest.Fallback):
        native_only(paths, 100)
    with pytest.raises((inputs.InputError, ValueError)) as want:
        inputs.load_inputs(*paths, 100, warn=None, native=False)
    with pytest.raises(type(want.value)) as got:
        inputs.load_inputs(*paths, 100, warn=None, native=True)
    assert str(got.value) == str(want.value)


@pytest.mark.parametrize("native", [True, False])
def test_ungrouped_blastout_keeps_every_run(tmp_path, native):
    """A contig whose hits come in two runs: both readers keep every hit in file order with
    its run number (regroup.py scores it run by run)."""
    first = BLAST.splitlines(True)[0]
    paths = _write(tmp_path, FNA, BLAST + first, GFF)
    if native:
        native_only(paths, 100)                           # (no fallback)
    b, _ = inputs.load_inputs(*paths, 100, warn=None, native=native)
    (tmp_path / "g").mkdir()
    grouped, _ = inputs.load_inputs(*_write(tmp_path / "g", FNA, BLAST, GFF), 100, warn=None,
                                    native=False)
    assert b.n_hits == grouped.n_hits + 1 and grouped.hit_group is None
    c = b.contig_names.index(first.split("\t", 1)[0])
    h0, h1 = int(b.hit_off[c]), int(b.hit_off[c + 1])
    assert b.hit_group[h0:h1].tolist() == [0] * (h1 - h0 - 1) + [1]
    assert int(b.hit_row[h1 - 1]) == len(BLAST.splitlines())
    assert not b.hit_group[:h0].any() and not b.hit_group[h1:].any()


def test_bad_rows_of_unknown_contigs_are_ignored(tmp_path):
    """The reference never builds hits of contigs missing from the FASTA, so their bad
    subject ids and zero lengths are not errors (orgscorer.py:944-946)."""
    blast = BLAST.replace("g3|s__Z|Q=z", "g3").replace(
        _row("c9", "g3"), _row("c9", "g3", slen=0).replace("\t0\t1\t300", "\t0\t1\t300"))
    paths = _write(tmp_path, FNA, blast, GFF)
    native_only(paths, 100)
    assert_same(*both(paths, 100))


def test_empty_inputs(tmp_path):
    paths = _write(tmp_path, "", "", "")
    a, b = both(paths, 100)
    assert_same(a, b)
    assert a[0].n_contigs == 0 and a[0].n_hits == 0


def test_dense_short_annotations_match(tmp_path):
    """Annotation items as short as "|=" (an empty system and value, utils.py:239-241): a
    row dense with them fills the annotation buffer at 2 bytes per item; the native parser
    must hold every one of them (a 4-byte-per-item reservation dropped them)."""
    dense = "g1|s__A" + "|=" * 400 + "|a=" * 50
    blast = _row("c1", dense) + _row("c1", "g2|s__B|=|=") + _row("c2", "g5|s__B" + "|=" * 300)
    paths = _write(tmp_path, FNA, blast, GFF)
    native_only(paths, 100)                            # the native path (no fallback)
    a, b = both(paths, 100)
    assert_same(a, b)
    assert a[0].systems == ["", "a"]


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_ungrouped_runs_across_chunks_native_equals_python(tmp_path, threads):
    """Runs of one contig in separate parts of a large file (several parse chunks), some
    split by a chunk boundary: the same hits, order and run numbers from both readers."""
    data = synth.generate(n=200, genes=6, clades=40, seed=17)
    paths = synth.write_text(data, str(tmp_path))
    lines = open(paths[1]).read().splitlines(True)
    by = {}
    for ln in lines:
        by.setdefault(ln.split("\t", 1)[0], []).append(ln)
    rounds = [[], [], []]
    for i, rows in enumerate(by.values()):
        k = 1 + i % 3
        for r in range(k):
            rounds[r].append(rows[r::k])
    with open(paths[1], "w") as fh:
        for rnd in rounds:
            for run in rnd:
                fh.writelines(run)
    a, b = both(paths, 200.0, threads=threads)
    assert_same(a, b)
    assert a[0].hit_group is not None and int(a[0].hit_group.max()) == 2
