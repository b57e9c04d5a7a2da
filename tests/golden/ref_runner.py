"""Run the REFERENCE waafle_orgscorer (build container only) and dump its decisions.

Usage: python ref_runner.py <mode> <dump.json> <orgscorer args...>

mode = "hash"   : the reference exactly as shipped (set order follows PYTHONHASHSEED)
mode = "sorted" : contig clade sets iterate in sorted name order -- one legal set
                  order, and the deterministic tie policy of this build.

Besides the normal TSVs (written by the reference itself), dumps per contig the
float64 bits (hex) of crit/rank of the final one- and two-clade options, their
clades, synteny and OK flag, and the final gene-score matrix, so the oracle and the
HIP path are pinned bit-for-bit, not just at the 4 printed decimals.

This script reads /root/reference, which exists only in the build container; it
is never run by the tests or on the GPU box.  Its outputs are the committed
fixtures next to it (see make_golden.py).
"""
import json
import os
import sys

REF = "/root/reference"


def main():
    mode, dump_path = sys.argv[1], sys.argv[2]
    sys.argv = ["waafle_orgscorer"] + sys.argv[3:]
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import waafle.waafle_orgscorer as ws  # noqa: E402

    if mode == "sorted":
        class SortedIterSet(set):
            def __iter__(self):
                return iter(sorted(set.__iter__(self)))

        upd, att = ws.Contig.update_gene_scores, ws.Contig.attach_hits

        def update_gene_scores(self):
            upd(self)
            self.clades = SortedIterSet(self.clades)

        def attach_hits(self, hits):
            att(self, hits)
            self.clades = SortedIterSet(self.clades)

        ws.Contig.update_gene_scores = update_gene_scores
        ws.Contig.attach_hits = attach_hits
    elif mode != "hash":
        raise SystemExit("bad mode " + mode)

    if "--write-details" in sys.argv:
        # --write-details raises on Python 3 upstream: try_open() hands print() a binary
        # GzipFile (utils.py:60-72, orgscorer.py:931-937).  Open that one file in text
        # mode; everything written to it is still the reference's own write_details().
        import gzip
        opener = ws.wu.try_open

        def try_open(path, *args):
            if path.endswith(".details.tsv.gz") and args == ("w",):
                return gzip.open(path, "wt")
            return opener(path, *args)

        ws.wu.try_open = try_open

    with_scores = os.environ.get("REF_DUMP_SCORES", "0") == "1"
    write = ws.write_main_output_files

    def write_main_output_files(contigs, taxonomy, args):
        dump = {}
        for name, C in contigs.items():
            rec = {}
            for tag, o in (("one", C.best_one), ("two", C.best_two)):
                if o is not None:
                    rec[tag] = [bool(o.ok), float(o.crit).hex(), float(o.rank).hex(),
                                o.clade1, o.clade2, o.synteny, o.direction]
            if with_scores:
                rec["S"] = {c: [float(x).hex() for x in v] for c, v in C.gene_scores.items()}
            dump[name] = rec
        with open(dump_path, "w") as fh:
            json.dump(dump, fh, sort_keys=True)
        write(contigs, taxonomy, args)

    ws.write_main_output_files = write_main_output_files
    ws.main()


if __name__ == "__main__":
    main()
