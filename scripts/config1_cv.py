"""Config 1: the reference's kernel/main.py sweep (10-fold CV of graph
classifiers on a TU dataset) on mgcn.  TU files are read from --root
(<root>/<NAME>_A.txt ...) when given, else the MUTAG-shaped synthetic set is
used (no download here).  Prints one JSON line with the result lines and the
wall time.

    python scripts/config1_cv.py --nets GCN GIN0 --layers 2 3 --hiddens 32 --epochs 100
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402

import mgcn.kernel as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--random_state", type=int, default=12345)
    ap.add_argument("--add_sl", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--lr", type=float, default=0.01)
    ap.add_argument("--lr_decay_factor", type=float, default=0.5)
    ap.add_argument("--lr_decay_step_size", type=int, default=50)
    ap.add_argument("--es_patience", type=int, default=-1)
    ap.add_argument("--folds", type=int, default=10)
    ap.add_argument("--datasets", nargs="+", default=["MUTAG"])
    ap.add_argument("--nets", nargs="+", default=["GCN"])
    ap.add_argument("--layers", nargs="+", type=int, default=[2])
    ap.add_argument("--hiddens", nargs="+", type=int, default=[32])
    ap.add_argument("--root", default=None, help="directory with the TU text files")
    args = ap.parse_args()
    random.seed(args.seed)
    torch.manual_seed(args.seed)
    t0 = time.perf_counter()
    lines = K.run_sweep(args.datasets, [getattr(K, n) for n in args.nets], args.layers,
                        args.hiddens, folds=args.folds, epochs=args.epochs,
                        batch_size=args.batch_size, lr=args.lr,
                        lr_decay_factor=args.lr_decay_factor,
                        lr_decay_step_size=args.lr_decay_step_size,
                        random_state=args.random_state, es_patience=args.es_patience,
                        add_sl=bool(args.add_sl), root=args.root,
                        synthetic=None if args.root else True, device=torch.device("cuda"))
    print(json.dumps({"workload": "config1 kernel/ 10-fold CV", "data": "TU files" if args.root
                      else "synthetic MUTAG-shaped", "results": lines,
                      "seconds": time.perf_counter() - t0}))


if __name__ == "__main__":
    main()
