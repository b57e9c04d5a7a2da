"""Seeded synthetic contig / hit / gene-call / taxonomy tables.

Shapes follow SURVEY.md §8(d) (BASELINE.json configs 2-5).  Everything is generated
as integer fields (pident in thousandths) so that the text rendering (BLAST
`-outfmt 6` with the 15 WAAFLE columns, utils.py:167-184; GFF, utils.py:282-292;
FASTA; 2-column taxonomy, utils.py:380) and the binary packing produce the SAME
float64 scores: `pident_milli / 1000.0` is the correctly rounded value of the
3-decimal string, exactly what `float("87.207")` returns.

Taxonomy: r__Root -> 1 k -> 2 p -> 4 c -> C/48 o -> C/16 f -> C/4 g -> C s, plus
1..3 t__ leaves per species (so leaf counts and sister sets are non-trivial).

Per contig: G genes (length U[250,1500), gap U[5,150), strand +/-).  Each gene gets
one full-length "owner" hit (pident U[85,100]) and D decoy hits from uniformly
drawn clades (pident U[70,90], 5 % U[80,100]; coverage U[0.8,1.0) at a random
offset).  A fraction `lgt_frac` of contigs carry a 2-gene run owned by a donor B.
The stress shape (`stress=True`, config 5) instead gives every other clade one
full-length hit on gene (clade mod G) with pident U(80.5,94.5), so ~C clades pass
the k2 pre-filter and the all-pairs search runs over ~C^2/2 pairs per contig.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

CONFIGS = {
    # name: (N contigs, G genes, C clades, extra)
    "demo": None,
    "cfg2": dict(n=10_000, genes=8, clades=200),
    "cfg3": dict(n=100_000, genes=12, clades=1000),
    "cfg4": dict(n=1_000_000, genes=10, clades=2000),
    "cfg5": dict(n=50_000, genes=20, clades=5000, stress=True),
}


@dataclass
class SynthTaxonomy:
    edges: list            # [(child, parent)] in file order
    species: list          # species names, index = clade number


@dataclass
class SynthData:
    tax: SynthTaxonomy
    contig_names: list
    contig_lengths: np.ndarray      # int64[N]
    # loci (grouped by contig, GFF order)
    loc_contig: np.ndarray          # int64[L]
    loc_start: np.ndarray           # int64[L]
    loc_end: np.ndarray             # int64[L]
    loc_strand: np.ndarray          # uint8[L]  (ord('+') / ord('-'))
    # hits (grouped by contig, sorted by qstart)
    hit_contig: np.ndarray          # int64[H]
    hit_clade: np.ndarray           # int64[H]  species index
    hit_gene: np.ndarray            # int64[H]  gene index (for the subject id)
    qlen: np.ndarray
    slen: np.ndarray
    length: np.ndarray
    qstart: np.ndarray
    qend: np.ndarray
    sstart: np.ndarray
    send: np.ndarray
    pident_milli: np.ndarray        # int64, pident * 1000
    minus: np.ndarray               # bool: sstrand == "minus"

    @property
    def n_contigs(self):
        return len(self.contig_names)

    @property
    def n_hits(self):
        return len(self.hit_contig)


def make_taxonomy(n_clades, rng):
    levels = [("k", 1), ("p", 2), ("c", 4), ("o", max(1, n_clades // 48)),
              ("f", max(1, n_clades // 16)), ("g", max(1, n_clades // 4)), ("s", n_clades)]
    edges = []
    prev = ["r__Root"]
    names_by_level = []
    for tag, count in levels:
        cur = ["{}__{}{}".format(tag, tag.upper(), i) for i in range(count)]
        for i, name in enumerate(cur):
            edges.append((name, prev[i * len(prev) // count]))
        names_by_level.append(cur)
        prev = cur
    species = names_by_level[-1]
    n_leaves = rng.integers(1, 4, size=n_clades)
    for i, sp in enumerate(species):
        for j in range(int(n_leaves[i])):
            edges.append(("t__S{}_{}".format(i, j), sp))
    return SynthTaxonomy(edges=edges, species=species)


def _subject_coords(aligned, extra, minus):
    """Subject coordinates for a fully aligned subject of length aligned+extra."""
    slen = aligned + extra
    sstart = np.where(minus, aligned, 1)
    send = np.where(minus, 1, aligned)
    return slen, sstart, send


def generate(n, genes, clades, decoys=20, lgt_frac=0.10, seed=0, stress=False,
             short_frac=0.0, name_prefix="contig"):
    rng = np.random.default_rng(seed)
    tax = make_taxonomy(clades, rng)
    return _generate_contigs(rng, tax, n, genes, clades, decoys, lgt_frac, stress, short_frac,
                             name_prefix, 0)


def _generate_contigs(rng, tax, n, genes, clades, decoys, lgt_frac, stress, short_frac,
                      name_prefix, first):
    """Contigs `first .. first + n - 1` drawn from `rng` (generate() draws the taxonomy
    from the same generator first; generate_chunk draws each chunk from its own)."""
    N, G = int(n), int(genes)

    glen = rng.integers(250, 1500, size=(N, G))
    if short_frac > 0:
        short = rng.random((N, G)) < short_frac
        glen = np.where(short, rng.integers(60, 200, size=(N, G)), glen)
    gap = rng.integers(5, 150, size=(N, G))
    gstart = np.cumsum(gap + np.concatenate([np.zeros((N, 1), np.int64), glen[:, :-1]], 1), 1) + 1
    gend = gstart + glen - 1
    gminus = rng.random((N, G)) < 0.5
    clen = gend[:, -1] + rng.integers(0, 150, size=N)

    owner = rng.integers(0, clades, size=N)
    donor = (owner + rng.integers(1, clades, size=N)) % clades if clades > 1 else owner
    has_lgt = np.ones(N, bool) if stress else rng.random(N) < lgt_frac
    run0 = rng.integers(0, max(1, G - 1), size=N)
    gidx = np.arange(G)[None, :]
    in_run = has_lgt[:, None] & (gidx >= run0[:, None]) & (gidx < run0[:, None] + 2)

    # owner hits: one per gene, full length
    o_clade = np.where(in_run, donor[:, None], owner[:, None])
    if stress:
        o_pid = np.where(in_run, rng.integers(90_000, 100_001, size=(N, G)),
                         rng.integers(85_000, 100_001, size=(N, G)))
    else:
        o_pid = rng.integers(85_000, 100_001, size=(N, G))
    o_minus = rng.random((N, G)) < 0.5
    o_slen, o_ss, o_se = _subject_coords(glen, rng.integers(0, 40, size=(N, G)), o_minus)
    parts = [dict(contig=np.repeat(np.arange(N), G), clade=o_clade.ravel(),
                  gene=np.tile(np.arange(G), N), qstart=gstart.ravel(), qend=gend.ravel(),
                  length=glen.ravel(), slen=o_slen.ravel(), sstart=o_ss.ravel(),
                  send=o_se.ravel(), pid=o_pid.ravel(), minus=o_minus.ravel())]

    if stress:
        # every other clade d: one full-length hit on gene d mod G
        d = np.arange(clades)
        per = []
        for i in range(N):
            keep = (d != owner[i]) & (d != donor[i] if has_lgt[i] else True)
            dd = d[keep]
            g = dd % G
            per.append((np.full(len(dd), i), dd, g))
        c_idx = np.concatenate([p[0] for p in per])
        c_cl = np.concatenate([p[1] for p in per])
        c_g = np.concatenate([p[2] for p in per])
        L = glen[c_idx, c_g]
        mi = rng.random(len(c_idx)) < 0.5
        sl, ss, se = _subject_coords(L, rng.integers(0, 40, size=len(c_idx)), mi)
        parts.append(dict(contig=c_idx, clade=c_cl, gene=c_g, qstart=gstart[c_idx, c_g],
                          qend=gend[c_idx, c_g], length=L, slen=sl, sstart=ss, send=se,
                          pid=rng.integers(80_501, 94_500, size=len(c_idx)), minus=mi))
    elif decoys > 0:
        M = N * G * decoys
        c_idx = np.repeat(np.arange(N), G * decoys)
        c_g = np.tile(np.repeat(np.arange(G), decoys), N)
        L = glen[c_idx, c_g]
        cov = rng.uniform(0.8, 1.0, size=M)
        a = np.maximum(1, (cov * L).astype(np.int64))
        off = (rng.random(M) * (L - a + 1)).astype(np.int64)
        qs = gstart[c_idx, c_g] + off
        hi = rng.random(M) < 0.05
        pid = np.where(hi, rng.integers(80_000, 100_001, size=M), rng.integers(70_000, 90_001, size=M))
        mi = rng.random(M) < 0.5
        sl, ss, se = _subject_coords(a, rng.integers(0, 40, size=M), mi)
        parts.append(dict(contig=c_idx, clade=rng.integers(0, clades, size=M), gene=c_g,
                          qstart=qs, qend=qs + a - 1, length=a, slen=sl, sstart=ss, send=se,
                          pid=pid, minus=mi))

    cat = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    order = np.lexsort((cat["qstart"], cat["contig"]))
    cat = {k: v[order] for k, v in cat.items()}

    names = ["{}{}".format(name_prefix, first + i) for i in range(N)]
    return SynthData(
        tax=tax, contig_names=names, contig_lengths=clen.astype(np.int64),
        loc_contig=np.repeat(np.arange(N), G), loc_start=gstart.ravel().astype(np.int64),
        loc_end=gend.ravel().astype(np.int64),
        loc_strand=np.where(gminus.ravel(), ord("-"), ord("+")).astype(np.uint8),
        hit_contig=cat["contig"].astype(np.int64), hit_clade=cat["clade"].astype(np.int64),
        hit_gene=cat["gene"].astype(np.int64), qlen=clen[cat["contig"]].astype(np.int64),
        slen=cat["slen"].astype(np.int64), length=cat["length"].astype(np.int64),
        qstart=cat["qstart"].astype(np.int64), qend=cat["qend"].astype(np.int64),
        sstart=cat["sstart"].astype(np.int64), send=cat["send"].astype(np.int64),
        pident_milli=cat["pid"].astype(np.int64), minus=cat["minus"].astype(bool))


CHUNK = 10_000     # contigs per independently seeded chunk (generate_chunk)
CHUNKS = {"cfg5": 500}   # stress contigs carry ~5000 hits each: smaller chunks


def chunk_size(name):
    return CHUNKS.get(name, CHUNK)


def chunk_taxonomy(name, seed=None):
    """Taxonomy of a chunked synthetic set: drawn from default_rng(seed) alone."""
    spec = CONFIGS[name]
    seed = int(name[-1]) if seed is None else seed
    return make_taxonomy(spec["clades"], np.random.default_rng(seed))


def generate_chunk(name, k, seed=None, tax=None, chunk=None, n_total=None):
    """Chunk k (contigs k*chunk .. ) of a BASELINE config drawn from its own generator
    default_rng([seed, k]) -- so any contig range is reproducible without generating
    the contigs before it, and chunks can be generated in parallel.  Same per-contig
    distributions as generate(); the taxonomy comes from chunk_taxonomy."""
    spec = dict(CONFIGS[name])
    seed = int(name[-1]) if seed is None else seed
    n_total = spec["n"] if n_total is None else n_total
    chunk = chunk_size(name) if chunk is None else chunk
    tax = chunk_taxonomy(name, seed) if tax is None else tax
    first = k * chunk
    n = min(chunk, n_total - first)
    rng = np.random.default_rng([seed, k])
    return _generate_contigs(rng, tax, n, spec["genes"], spec["clades"], 20, 0.10,
                             spec.get("stress", False), 0.0, "contig", first)


def _pack_chunk(args):
    """Worker: chunk k -> the device arrays of its contigs (no names, no annotation text)."""
    name, k, seed, chunk, n_total = args
    d = generate_chunk(name, k, seed, chunk=chunk, n_total=n_total)
    from .inputs import derive_hit_values
    scov, score = derive_hit_values(d.qlen, d.slen, d.qstart, d.qend, d.sstart, d.send,
                                    d.pident_milli / 1000.0, d.minus)
    keep = (np.abs(d.loc_end - d.loc_start) + 1) >= 200.0
    return dict(
        hit_cnt=np.bincount(d.hit_contig, minlength=d.n_contigs).astype(np.int64),
        loc_cnt=np.bincount(d.loc_contig[keep], minlength=d.n_contigs).astype(np.int64),
        hit_qlo=np.minimum(d.qstart, d.qend).astype(np.int32),
        hit_qhi=np.maximum(d.qstart, d.qend).astype(np.int32),
        hit_clade=d.hit_clade.astype(np.int32), hit_strand=d.minus.astype(np.int8),
        hit_score=score, hit_scov=scov,
        loc_start=d.loc_start[keep].astype(np.int32), loc_end=d.loc_end[keep].astype(np.int32),
        loc_strand=np.where(d.loc_strand[keep] == ord("-"), 1, 0).astype(np.int8),
        contig_lengths=d.contig_lengths)


def generate_batch(name, lo=0, hi=None, seed=None, workers=None, chunk=None, n_total=None):
    """Contigs [lo, hi) of a BASELINE config (whole chunks) packed straight into a device
    batch, chunks generated in parallel worker processes.  Returns (HostBatch,
    TaxonomyTables).  The batch carries no contig names or annotation values (the bench
    never renders TSVs); every hit has annotation system 0 (sysmask 1), as to_batch."""
    from .inputs import HostBatch
    from .taxonomy import TaxonomyTables
    spec = CONFIGS[name]
    n_total = spec["n"] if n_total is None else n_total
    chunk = chunk_size(name) if chunk is None else chunk
    hi = n_total if hi is None else hi
    seed = int(name[-1]) if seed is None else seed
    st = make_taxonomy(spec["clades"], np.random.default_rng(seed))
    tax = TaxonomyTables(st.edges)
    clade_to_id = np.array([tax.index[sp] for sp in st.species], dtype=np.int32)
    ks = list(range(lo // chunk, (hi + chunk - 1) // chunk))
    jobs = [(name, k, seed, chunk, n_total) for k in ks]
    if workers is None:
        workers = min(16, len(os.sched_getaffinity(0)), len(jobs))
    if workers > 1:
        import multiprocessing as mp
        # close + join, not the context manager's terminate(): SIGTERM'd workers hang in an
        # attached profiler's signal handler (rocprofv3), and the parent waits on them
        pool = mp.get_context("fork").Pool(workers)
        try:
            parts = pool.map(_pack_chunk, jobs, chunksize=1)
        finally:
            pool.close()
            pool.join()
    else:
        parts = [_pack_chunk(j) for j in jobs]
    # trim to [lo, hi)
    c0 = lo - ks[0] * chunk
    n = hi - lo
    cat = lambda f: np.concatenate([p[f] for p in parts])
    hit_cnt, loc_cnt = cat("hit_cnt"), cat("loc_cnt")
    hoff = np.concatenate([[0], np.cumsum(hit_cnt)])
    loff = np.concatenate([[0], np.cumsum(loc_cnt)])
    ha, hb = int(hoff[c0]), int(hoff[c0 + n])
    la, lb = int(loff[c0]), int(loff[c0 + n])
    hit_off = (hoff[c0:c0 + n + 1] - ha).astype(np.int64)
    loc_off = (loff[c0:c0 + n + 1] - la).astype(np.int64)

    def hits(f):
        return np.concatenate([p[f] for p in parts])[ha:hb]

    batch = HostBatch(
        contig_names=[], contig_lengths=cat("contig_lengths")[c0:c0 + n],
        hit_off=hit_off, hit_qlo=hits("hit_qlo"), hit_qhi=hits("hit_qhi"),
        hit_taxon=clade_to_id[hits("hit_clade")], hit_strand=hits("hit_strand"),
        hit_score=hits("hit_score"), hit_scov=hits("hit_scov"),
        hit_sysmask=np.ones(hb - ha, dtype=np.uint32), loc_off=loc_off,
        loc_start=cat("loc_start")[la:lb], loc_end=cat("loc_end")[la:lb],
        loc_strand=cat("loc_strand")[la:lb], systems=["UniProt"])
    return batch, tax


def generate_config(name, seed=None, n=None, **kw):
    spec = dict(CONFIGS[name])
    if n is not None:
        spec["n"] = n
    spec.update(kw)
    return generate(seed=(int(name[-1]) if seed is None else seed), **spec)


# ---------------------------------------------------------------------------
# text rendering (the reference's on-disk formats)
# ---------------------------------------------------------------------------

def sseqids(data):
    sp = data.tax.species
    return ["GENE{}_{}|{}|UniProt=U{}x{}".format(c, g, sp[c], c, g % 50)
            for c, g in zip(data.hit_clade.tolist(), data.hit_gene.tolist())]


def write_text(data, outdir, basename="synth"):
    """Write <basename>.fna / .blastout / .gff / .taxonomy.tsv; returns the 4 paths."""
    os.makedirs(outdir, exist_ok=True)
    paths = [os.path.join(outdir, basename + ext)
             for ext in (".fna", ".blastout", ".gff", ".taxonomy.tsv")]
    with open(paths[0], "w") as fh:
        for name, n in zip(data.contig_names, data.contig_lengths.tolist()):
            fh.write(">{}\n".format(name))
            for i in range(0, n, 80):
                fh.write("N" * min(80, n - i) + "\n")
    names = data.contig_names
    sids = sseqids(data)
    pm = data.pident_milli
    pid = ["{}.{:03d}".format(v // 1000, v % 1000) for v in pm.tolist()]
    cols = [data.hit_contig.tolist(), sids, data.qlen.tolist(), data.slen.tolist(),
            data.length.tolist(), data.qstart.tolist(), data.qend.tolist(),
            data.sstart.tolist(), data.send.tolist(), pid,
            ((data.length * pm) // 100_000).tolist(), data.minus.tolist()]
    with open(paths[1], "w") as fh:
        for (ci, sid, ql, sl, ln, qs, qe, ss, se, pi, pos, mi) in zip(*cols):
            fh.write("{}\t{}\t{}\t{}\t{}\t{}\t{}\t{}\t{}\t{}\t{}\t0\t0.0\t{}\t{}\n".format(
                names[ci], sid, ql, sl, ln, qs, qe, ss, se, pi, pos, ln * 2,
                "minus" if mi else "plus"))
    with open(paths[2], "w") as fh:
        fh.write("##gff-version 3\n")
        for ci, s, e, st in zip(data.loc_contig.tolist(), data.loc_start.tolist(),
                                data.loc_end.tolist(), data.loc_strand.tolist()):
            fh.write("{}\tsynth\tgene\t{}\t{}\t.\t{}\t0\t.\n".format(names[ci], s, e, chr(st)))
    with open(paths[3], "w") as fh:
        for child, parent in data.tax.edges:
            fh.write("{}\t{}\n".format(child, parent))
    return paths


# ---------------------------------------------------------------------------
# direct packing (identical arrays to parsing the text rendering)
# ---------------------------------------------------------------------------

def to_batch(data, min_gene_length=200.0, with_codes=True):
    """SynthData -> (HostBatch, TaxonomyTables) without going through text files."""
    from .inputs import HostBatch, derive_hit_values
    from .taxonomy import TaxonomyTables

    sp = data.tax.species
    used = np.unique(data.hit_clade)
    tax = TaxonomyTables(data.tax.edges, extra_names={sp[int(c)] for c in used})
    clade_to_id = np.full(len(sp), -1, dtype=np.int32)
    for c in used.tolist():
        clade_to_id[c] = tax.index[sp[c]]
    N = data.n_contigs
    hit_off = np.zeros(N + 1, dtype=np.int64)
    np.cumsum(np.bincount(data.hit_contig, minlength=N), out=hit_off[1:])
    pident = data.pident_milli / 1000.0
    scov, score = derive_hit_values(data.qlen, data.slen, data.qstart, data.qend, data.sstart,
                                    data.send, pident, data.minus)
    keep = (np.abs(data.loc_end - data.loc_start) + 1) >= min_gene_length
    loc_contig = data.loc_contig[keep]
    loc_off = np.zeros(N + 1, dtype=np.int64)
    np.cumsum(np.bincount(loc_contig, minlength=N), out=loc_off[1:])
    ls, le, lst = data.loc_start[keep], data.loc_end[keep], data.loc_strand[keep]
    codes = []
    if with_codes:
        codes = ["{}:{}:{}".format(a, b, chr(c)) for a, b, c in
                 zip(ls.tolist(), le.tolist(), lst.tolist())]
    # one annotation system ("UniProt"), value "U<clade>x<gene mod 50>", interned in
    # first-appearance order like the parser does
    vkey = data.hit_clade * 50 + data.hit_gene % 50
    uniq, first, inv = np.unique(vkey, return_index=True, return_inverse=True)
    rank = np.empty(len(uniq), dtype=np.int32)
    rank[np.argsort(first, kind="stable")] = np.arange(len(uniq), dtype=np.int32)
    value_ids = rank[inv].reshape(-1, 1).astype(np.int32)
    values = [None] * len(uniq)
    for k, u in zip(rank.tolist(), uniq.tolist()):
        values[k] = "U{}x{}".format(u // 50, u % 50)
    batch = HostBatch(
        contig_names=list(data.contig_names), contig_lengths=data.contig_lengths.copy(),
        hit_off=hit_off, hit_qlo=np.minimum(data.qstart, data.qend).astype(np.int32),
        hit_qhi=np.maximum(data.qstart, data.qend).astype(np.int32),
        hit_taxon=clade_to_id[data.hit_clade], hit_strand=data.minus.astype(np.int8),
        hit_score=score, hit_scov=scov, hit_sysmask=np.ones(data.n_hits, dtype=np.uint32),
        loc_off=loc_off, loc_start=ls.astype(np.int32), loc_end=le.astype(np.int32),
        loc_strand=np.where(lst == ord("-"), 1, np.where(lst == ord("+"), 0, 2)).astype(np.int8),
        loc_codes=codes, systems=["UniProt"], annot_value_ids=value_ids,
        annot_values=[values], hit_row=np.arange(data.n_hits, dtype=np.int64))
    return batch, tax


def _write_chunk(args):
    """Worker: chunk k of a chunked config rendered as text part files."""
    name, k, outdir = args
    write_text(generate_chunk(name, k), outdir, "part{:06d}".format(k))
    return k


def write_text_chunked(name, outdir, basename="synth", workers=None):
    """Text rendering of a whole chunked config (the 4 files of write_text), its chunks
    generated and written in parallel worker processes and concatenated in contig order.
    Returns (paths, contigs, hits)."""
    import shutil
    spec = CONFIGS[name]
    chunk = chunk_size(name)
    ks = list(range((spec["n"] + chunk - 1) // chunk))
    parts = os.path.join(outdir, basename + ".parts")
    os.makedirs(parts, exist_ok=True)
    if workers is None:
        workers = min(16, len(os.sched_getaffinity(0)), len(ks))
    jobs = [(name, k, parts) for k in ks]
    if workers > 1:
        import multiprocessing as mp
        pool = mp.get_context("fork").Pool(workers)     # close + join (see generate_batch)
        try:
            pool.map(_write_chunk, jobs, chunksize=1)
        finally:
            pool.close()
            pool.join()
    else:
        for j in jobs:
            _write_chunk(j)
    exts = (".fna", ".blastout", ".gff", ".taxonomy.tsv")
    paths = [os.path.join(outdir, basename + e) for e in exts]
    hits = 0
    for e, dest in zip(exts, paths):
        srcs = [os.path.join(parts, "part{:06d}{}".format(k, e)) for k in ks]
        if e == ".taxonomy.tsv":
            srcs = srcs[:1]                       # every chunk shares the config's taxonomy
        with open(dest, "wb") as out:
            for src in srcs:
                with open(src, "rb") as fh:
                    if e == ".blastout":
                        data = fh.read()
                        hits += data.count(b"\n")
                        out.write(data)
                    else:
                        shutil.copyfileobj(fh, out)
    shutil.rmtree(parts)
    return paths, spec["n"], hits
