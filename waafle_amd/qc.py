"""`waafle_qc` drop-in (waafle_qc.py:133-192): keeps the `.lgt.tsv` rows whose AB/BA
junctions are supported by read pairs or by coverage.

    python -m waafle_amd.qc contigs.lgt.tsv contigs.junctions.tsv [--outfile PATH]

A row passes when every adjacent locus pair with synteny AB or BA (LOCI and SYNTENY are
read from the orgscorer row, :169-183) has junction hits >= --min-junction-hits or a
coverage ratio >= --min-junction-ratio in the waafle_junctions table (keyed by the two
locus codes, :141-148).  A few hundred rows of table lookups: host code; the junction
table itself comes from the MI355X path (waafle_amd.junctions).
"""
import argparse
import csv
import sys

from .inputs import say


def build_parser():
    ap = argparse.ArgumentParser(description="waafle_qc: applies junction results to QC "
                                             "WAAFLE calls", formatter_class=argparse.RawTextHelpFormatter)
    g = ap.add_argument_group("required inputs")
    g.add_argument("contig_profile", help="lgt output from waafle_orgscorer (tsv format)")
    g.add_argument("junctions", help="output from waafle_junctions for contigs of interest")
    g = ap.add_argument_group("filtering parameters")
    g.add_argument("--min-junction-hits", type=int, default=2, metavar="<int>",
                   help="minimum read-hits to 'ok' a junction\n[default: 2]")
    # type=int with a float default, as upstream (:86-92): only integers parse on the CLI
    g.add_argument("--min-junction-ratio", type=int, default=0.5, metavar="<float>",
                   help="minimum coverage (relative to flanking genes) to 'ok' a junction\n[default: 0.5]")
    g = ap.add_argument_group("misc options")
    g.add_argument("--outfile", type=str, default=None, metavar="<path>",
                   help="Path for filtered outputs\n[default: derive from input]")
    return ap


def _frame(path):
    fh = open(path)
    reader = csv.reader(fh, dialect="excel-tab")
    return fh, next(reader), reader


def load_junctions(path):
    """{contig: {(gene1, gene2): hits}}, {contig: {(gene1, gene2): ratio}} (:137-148)."""
    hits, covs = {}, {}
    fh, headers, reader = _frame(path)
    with fh:
        for row in reader:
            R = dict(zip(headers, row))
            key = (R["GENE1"], R["GENE2"])
            hits.setdefault(R["CONTIG"], {})[key] = int(R["JUNCTION_HITS"])
            covs.setdefault(R["CONTIG"], {})[key] = float(R["RATIO"])
    return hits, covs


def passes(R, hits, covs, min_hits, min_ratio):
    """The per-row test (:169-183); None when the contig has no junction data."""
    contig = R["CONTIG_NAME"]
    if contig not in hits or contig not in covs:
        return None
    loci = R["LOCI"].split("|")
    syn = R["SYNTENY"]
    ok = True
    for i in range(len(loci) - 1):
        if syn[i] + syn[i + 1] not in ("AB", "BA"):
            continue
        pair = (loci[i], loci[i + 1])
        ok = ok and (hits[contig].get(pair, -1) >= min_hits or covs[contig].get(pair, -1) >= min_ratio)
    return ok


def main(argv=None):
    args = build_parser().parse_args(argv)
    say("Loading junctions report.")
    hits, covs = load_junctions(args.junctions)
    outfile = args.outfile if args.outfile is not None else args.contig_profile + ".qc_pass"
    total = failed = 0
    fh, headers, reader = _frame(args.contig_profile)
    with fh, open(outfile, "w") as out:
        out.write("\t".join(h.upper() for h in headers) + "\n")
        for row in reader:
            R = dict(zip(headers, row))
            if set(R) != set(headers):
                say("LETHAL ERROR: Format mismatch.")
                sys.exit("EXITING.")
            total += 1
            ok = passes(R, hits, covs, args.min_junction_hits, args.min_junction_ratio)
            if ok is None:
                failed += 1
                say("Missing junction data for contig:", R["CONTIG_NAME"])
            elif not ok:
                failed += 1
                say("Failed QC:", R["CONTIG_NAME"])
            else:
                out.write("\t".join(R[h] if R[h] != "" else "--" for h in headers) + "\n")
    say("Failure rate: {} of {} ({:.1f}%)".format(failed, total, 100 * failed / float(total)))
    say("Finished successfully.")


if __name__ == "__main__":
    main()
