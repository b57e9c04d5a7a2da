"""`waafle_orgscorer` command-line surface (drop-in).

Same positionals, flags, choices, defaults and types as the reference
(`waafle/waafle_orgscorer.py:135-303` plus the shared gene-caller arguments at
`waafle/waafle_genecaller.py:81-101`), plus one addition that the reference does
not have: `--gpus` (how many devices to shard contigs over; default 1).
"""

import argparse

DESCRIPTION = """\
waafle_orgscorer (MI355X build): Step 2 in the WAAFLE pipeline

Merges blast hits into genes on contigs-of-interest. Uses corresponding
taxonomy file, and the WAAFLE algorithm, to identify contigs that are
best explained by a single clade vs. a pair of clades. The latter events
correspond to putative LGTs. Contig scoring runs as HIP kernels on AMD
Instinct MI355X (gfx950)."""


def build_parser():
    parser = argparse.ArgumentParser(description=DESCRIPTION,
                                     formatter_class=argparse.RawTextHelpFormatter)
    g = parser.add_argument_group("required inputs")
    g.add_argument("contigs", help="contigs file (.fasta format)")
    g.add_argument("blastout", help="output of waafle_search for one set of contigs (.blastout)")
    g.add_argument("gff", help="gene calls (from waafle_genecaller or user-supplied) for <contigs> (.gff)")
    g.add_argument("taxonomy", help="taxonomy file for the blast database used to make <blastout>")

    g = parser.add_argument_group("output formatting")
    g.add_argument("--outdir", default=".", metavar="<path>",
                   help="directory for writing output files\n[default: .]")
    g.add_argument("--basename", default=None, metavar="<str>",
                   help="basename for output files\n[default: derived from contigs file]")
    g.add_argument("--write-details", action="store_true",
                   help="make an additional output file with per-gene clade scores\n[default: off]")
    g.add_argument("--quiet", action="store_true", help="don't show running progress\n[default: off]")

    g = parser.add_argument_group("main parameters")
    g.add_argument("-k1", "--one-clade-threshold", type=float, default=0.5, metavar="<0.0-1.0>",
                   help="minimum per-gene score for explaining a contig with a single clade\n[default: 0.5]")
    g.add_argument("-k2", "--two-clade-threshold", type=float, default=0.8, metavar="<0.0-1.0>",
                   help="minimum per-gene score for explaining a contig with a pair of clades (putative LGT)\n[default: 0.8]")
    g.add_argument("--disambiguate-one", choices=["report-best", "meld"], default="meld",
                   metavar="<report-best/meld>",
                   help="what to do when other one-clade explanations fall within <--range> of the best explanation\n[default: meld]")
    g.add_argument("--disambiguate-two", choices=["report-best", "jump", "meld"], default="meld",
                   metavar="<report-best/jump/meld>",
                   help="what to do when other two-clade explanations fall within <--range> of the best explanation\n[default: meld]")
    g.add_argument("--range", type=float, default=0.05, metavar="<float>",
                   help="when disambiguating, consider explanations within <--range> of the best explanation\n[default: 0.05]")
    g.add_argument("--jump-taxonomy", type=int, default=None, metavar="<1-N>",
                   help="before starting, perform 1+ 'jumps' up the taxonomy (e.g. species->genus)\n[default: off]")

    g = parser.add_argument_group("post-detection LGT filters")
    g.add_argument("--allow-lca", action="store_true",
                   help="when melding LGT clades, allow the LGT LCA to occur as a melded clade\n[default: off]")
    g.add_argument("--ambiguous-fraction", type=float, default=0.1, metavar="<0.0-1.0>",
                   help="allowed fraction of ambiguous (A OR B) gene length in a putative A+B contig\n[default: 0.1]")
    g.add_argument("--ambiguous-threshold", choices=["off", "lenient", "strict"], default="lenient",
                   metavar="<off/lenient/strict>",
                   help="homology threshold for defining an ambiguous (A OR B) gene\n[default: lenient]")
    g.add_argument("--sister-penalty", choices=["off", "lenient", "strict"], default="strict",
                   metavar="<off/lenient/strict>",
                   help="penalize homologs of missing genes in sisters of LGT clades (or just recipient if known)\n[default: strict]")
    g.add_argument("--clade-genes", type=int, default=None, metavar="<1-N>",
                   help="required minimum genes assigned to each LGT clade\n[default: off]")
    g.add_argument("--clade-leaves", type=int, default=None, metavar="<1-N>",
                   help="required minimum leaf count supporting each LGT clade (or just recipient if known)\n[default: off]")

    g = parser.add_argument_group("gene-hit merge parameters")
    g.add_argument("--weak-loci", choices=["ignore", "penalize", "assign-unknown"], default="ignore",
                   metavar="<ignore/penalize/assign-unknown>",
                   help="method for handling loci that are never assigned to known clades\n[default: ignore]")
    g.add_argument("--annotation-threshold", choices=["off", "lenient", "strict"], default="lenient",
                   metavar="<off/lenient/strict>",
                   help="stringency of gene annotation transfer to loci\n[default: lenient]")
    g.add_argument("--min-overlap", type=float, default=0.1, metavar="<0.0-1.0>",
                   help="only merge hits into genes if the longer of the two covers this portion of the shorter\n[default: 0.1]")
    # shared with waafle_genecaller (genecaller.py:81-101); --min-gene-length is a float upstream
    g.add_argument("--min-gene-length", default=200, type=float, metavar="<int>",
                   help="minimum allowed gene length\n[default: 200]")
    g.add_argument("--min-scov", default=0.75, type=float, metavar="<float>",
                   help="(modified) scoverage filter for hits to gene catalog\n[default: 0.75]")
    g.add_argument("--stranded", action="store_true",
                   help="only merge hits into hits/genes of the same strandedness\n[default: off]")

    g = parser.add_argument_group("MI355X execution")
    g.add_argument("--gpus", type=int, default=1, metavar="<1-8>",
                   help="number of GPUs to shard contigs over (one HIP context per device)\n[default: 1]")
    return parser


PARAM_KEYS = ("one_clade_threshold", "two_clade_threshold", "disambiguate_one", "disambiguate_two",
              "range", "jump_taxonomy", "allow_lca", "ambiguous_fraction", "ambiguous_threshold",
              "sister_penalty", "clade_genes", "clade_leaves", "weak_loci", "annotation_threshold",
              "min_overlap", "min_gene_length", "min_scov", "stranded")


def parse_flags(flags, positionals=("c", "b", "g", "t")):
    """Parse just the option flags (for tests / programmatic use)."""
    return build_parser().parse_args(list(positionals) + list(flags))


def param_dict(args):
    return {k: getattr(args, k) for k in PARAM_KEYS}
