"""`waafle_orgscorer` drop-in CLI (orgscorer.py:900-966) running on MI355X.

    python -m waafle_amd.orgscorer contigs.fna hits.blastout genes.gff taxonomy.tsv [flags]

Writes <basename>.lgt.tsv / .no_lgt.tsv / .unclassified.tsv exactly as the reference.
"""
import os
import sys
import time

from . import cli, engine, inputs, lib, output, regroup
from . import details as wdetails
from . import dist as wdist


def die(*args):
    inputs.say(*(["LETHAL ERROR:"] + list(args)))
    sys.exit("EXITING.")


def main(argv=None):
    args = cli.build_parser().parse_args(argv)
    say = (lambda *a: None) if args.quiet else inputs.say
    rank, world, local = wdist.rank_env()
    group = None
    if world > 1:
        # launched by torch.distributed.run: one process per GPU.  The inputs are parsed once,
        # on rank 0, which sends every rank its contig range as typed arrays (host to host:
        # gloo -- there is no device-side exchange); WAAFLE_DEVICE_MAP (e.g. "0,0") places
        # the ranks on devices other than their local rank (a rehearsal on one GPU)
        import torch.distributed as group
        group.init_process_group("gloo")
    dmap = os.environ.get("WAAFLE_DEVICE_MAP")
    device = int(dmap.split(",")[local]) if dmap else local
    t0 = time.time()
    batch = tax = None
    load_err = None
    if rank == 0:
        say("Loading inputs.")
        try:
            batch, tax = inputs.load_inputs(args.contigs, args.blastout, args.gff, args.taxonomy,
                                            args.min_gene_length, warn=inputs.say)
        except (inputs.InputError, ValueError) as exc:
            load_err = exc
    if group is not None:                  # every rank learns of rank 0's failure first
        load_err = wdist.share_error(load_err, group)
    if load_err is not None:
        if group is not None:
            group.destroy_process_group()
        if rank == 0:
            die(str(load_err))
        sys.exit("EXITING.")
    if rank == 0:
        if args.basename is None:
            args.basename = inputs.basename_of(args.contigs)
        say("Analyzing {:,} contigs ({:,} hits, {:,} loci) on {} GPU(s).".format(
            batch.n_contigs, batch.n_hits, batch.n_loci, world if group is not None else args.gpus))
    t1 = time.time()
    det = None
    try:
        if args.write_details:
            # per-level records come from one context (a diagnostic output: one GPU)
            if group is not None or args.gpus != 1:
                die("--write-details runs on one GPU (--gpus 1, no torch.distributed launch)")
            scorer = engine.GpuScorer(0)
            try:
                scorer.set_taxonomy(tax)
                res, det = scorer.score_details(batch, cli.param_dict(args))
            finally:
                scorer.close()
        elif group is None:
            res = engine.score(batch, tax, cli.param_dict(args), gpus=args.gpus)
        else:
            pre_err = None
            if rank == 0 and batch.hit_group is not None:
                # an ungrouped blastout: the earlier runs' evaluations on rank 0, the ranks
                # then score the batch of raised clades (regroup.py)
                try:
                    scorer = engine.GpuScorer(device)
                    try:
                        scorer.set_taxonomy(tax)
                        params = cli.param_dict(args)
                        batch = regroup.resolve(batch, tax.parent, params, lambda b: scorer.score(b, params))
                    finally:
                        scorer.close()
                except lib.WaafleHipError as exc:
                    pre_err = exc
            pre_err = wdist.share_error(pre_err, group)
            if pre_err is not None:
                raise pre_err

            def score_shard(sub, stax, a, b):
                inputs.say("  rank {}: contigs {}..{} ({:,} hits) on device {}".format(
                    rank, a, b, sub.n_hits, device))
                scorer = engine.GpuScorer(device)
                try:
                    scorer.set_taxonomy(stax)
                    return scorer.score(sub, cli.param_dict(args))
                finally:
                    scorer.close()
            res = wdist.score_ranked(batch, tax, cli.param_dict(args), score_shard, group)
    except lib.WaafleHipError as exc:
        if group is not None:
            group.destroy_process_group()
        if exc.code == lib.WF_E_RUNAWAY and len(getattr(exc, "contigs", ())):
            if rank == 0:
                die("  Warning: Runaway taxonomic recursion for",
                    batch.contig_names[int(exc.contigs[0])])
            sys.exit("EXITING.")
        die(str(exc))
    t2 = time.time()
    if group is not None:
        group.destroy_process_group()
        if rank != 0:
            return
    if det is not None:
        try:
            wdetails.write(wdetails.render(batch, tax, cli.param_dict(args), det),
                           args.outdir, args.basename)
        except wdetails.DetailsError as exc:
            die(str(exc))
    say("Initializing outputs.")
    rows = output.render(batch, tax, res)
    output.write(rows, args.outdir, args.basename)
    say("Finished successfully (parse {:.2f}s, score {:.3f}s, write {:.2f}s).".format(
        t1 - t0, t2 - t1, time.time() - t2))


if __name__ == "__main__":
    main()
