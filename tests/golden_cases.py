"""Loading committed golden fixtures and materialising their inputs (no reference access)."""
import glob
import gzip
import json
import os
import shutil

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
DEMO_FILES = {
    "homology": ["demo_contigs.fna", "demo_contigs.blastout", "demo_contigs.gff", "demo_taxonomy.tsv"],
    "prodigal": ["demo_contigs.fna", "demo_contigs.blastout", "demo_contigs.prodigal.gff",
                 "demo_taxonomy.tsv"],
}


def case_names():
    return sorted(os.path.basename(p)[:-len(".json.gz")]
                  for p in glob.glob(os.path.join(GOLDEN, "*.json.gz"))
                  if not os.path.basename(p).startswith("details_")
                  and ".runaway." not in os.path.basename(p)
                  and ".junc." not in os.path.basename(p))


# fixtures whose explain_two is too large for the scalar oracle (cfg5 stress contigs:
# 12.5 M clade pairs each): the HIP path is compared with the reference-generated fixture
# (TSVs + decision dump) only, never with a re-run oracle
HEAVY = {"syn_cfg5_default"}


def runaway_names():
    """Deep-taxonomy fixtures (make_deep.py): reference TSVs or its runaway die."""
    return sorted(os.path.basename(p)[:-len(".runaway.json.gz")]
                  for p in glob.glob(os.path.join(GOLDEN, "*.runaway.json.gz")))


def load_runaway(name):
    with gzip.open(os.path.join(GOLDEN, name + ".runaway.json.gz"), "rt") as fh:
        return json.load(fh)


def details_names():
    """--write-details fixtures (make_details.py)."""
    return sorted(os.path.basename(p)[:-len(".json.gz")]
                  for p in glob.glob(os.path.join(GOLDEN, "details_*.json.gz")))


def load(name):
    with gzip.open(os.path.join(GOLDEN, name + ".json.gz"), "rt") as fh:
        return json.load(fh)


def demo_file(fname, tmpdir):
    dest = os.path.join(str(tmpdir), fname)
    if not os.path.exists(dest):
        with gzip.open(os.path.join(GOLDEN, "demo_inputs", fname + ".gz"), "rb") as src, \
                open(dest, "wb") as out:
            shutil.copyfileobj(src, out)
    return dest


def materialize(fixture, tmpdir):
    """Return the 4 input paths (contigs, blastout, gff, taxonomy) for a fixture."""
    recipe = fixture["recipe"]
    if recipe["kind"] == "demo":
        return [demo_file(f, tmpdir) for f in DEMO_FILES[recipe["gff"]]]
    if recipe["kind"] == "files":
        d = os.path.join(GOLDEN, recipe["dir"])
        stem = recipe.get("stem", "tie")
        return [os.path.join(d, stem + e) for e in
                (".fna", ".blastout", ".gff", ".taxonomy.tsv")]
    from waafle_amd import synth
    sub = os.path.join(str(tmpdir), "synth_" + "_".join(
        "{}{}".format(k, v) for k, v in sorted(recipe["params"].items())))
    paths = [os.path.join(sub, "synth" + e) for e in (".fna", ".blastout", ".gff", ".taxonomy.tsv")]
    if not os.path.exists(paths[-1]):
        synth.write_text(synth.generate(**recipe["params"]), sub, "synth")
    return paths


def rows_by_contig(texts):
    out = {}
    for kind, text in texts.items():
        for line in text.splitlines()[1:]:
            out[line.split("\t", 1)[0]] = (kind, line)
    return out


def headers(texts):
    return {kind: text.splitlines()[0] for kind, text in texts.items()}


def compare_tsv(fixture, texts):
    """Compare produced TSV texts {kind: text} with a fixture; tie contigs may match any
    of the reference's outcomes.  Returns a list of mismatch descriptions."""
    bad = []
    want_h, got_h = headers(fixture["tsv"]), headers(texts)
    if want_h != got_h:
        bad.append(("headers", want_h, got_h))
    want, got = rows_by_contig(fixture["tsv"]), rows_by_contig(texts)
    if set(want) != set(got):
        bad.append(("contig set", sorted(set(want) ^ set(got))[:10]))
    for contig, row in want.items():
        g = got.get(contig)
        if g == row:
            continue
        if contig in fixture["ties"] and g is not None and list(g) in fixture["alt_rows"].get(contig, []):
            continue
        bad.append((contig, row, g))
    for kind, text in fixture["tsv"].items():   # row order (sorted contig names)
        order_w = [l.split("\t", 1)[0] for l in text.splitlines()[1:]]
        order_g = [l.split("\t", 1)[0] for l in texts[kind].splitlines()[1:]]
        if order_w != order_g:
            bad.append(("row order", kind))
    return bad


def junction_names():
    """waafle_junctions / waafle_qc fixtures (make_junctions.py)."""
    return sorted(os.path.basename(p)[:-len(".junc.json.gz")]
                  for p in glob.glob(os.path.join(GOLDEN, "*.junc.json.gz")))


def load_junction(name):
    with gzip.open(os.path.join(GOLDEN, name + ".junc.json.gz"), "rt") as fh:
        return json.load(fh)


def materialize_junction(fixture, tmpdir):
    """(fna, gff, sam, lgt.tsv) paths for a junction fixture, rebuilt from its recipe."""
    from waafle_amd import synth, synth_reads
    r = fixture["recipe"]
    sub = os.path.join(str(tmpdir), "junc_" + "_".join(
        "{}{}".format(k, v) for k, v in sorted(r["generate"].items())))
    fna, gff = os.path.join(sub, "synth.fna"), os.path.join(sub, "synth.gff")
    sam, lgt = os.path.join(sub, "reads.sam"), os.path.join(sub, "synth.lgt.tsv")
    if not os.path.exists(lgt):
        data = synth.generate(**r["generate"])
        synth.write_text(data, sub, "synth")
        synth_reads.write_sam(data, sam, **r["reads"])
        with open(lgt, "w") as fh:
            fh.write(load(r["lgt_golden"])["tsv"]["lgt"])
    return fna, gff, sam, lgt
