"""Config 3 end to end: src/run/train_botnet.py on mgcn (GCNModel, CE or
focal loss, Adam + ReduceLROnPlateau + early stopping, per-graph metrics).
Data: --data_dir with .npz files (mgcn.botnet layout; see
scripts/botnet_h5_to_npz.py), or synthetic config-3-shaped graphs when no
files are given.  Prints one JSON line with the history.

    python scripts/train_botnet.py --enc_sizes 32 32 32 32 32 32 32 32 32 32 32 32 \
        --residual_hop 1 --epochs 3
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]
import torch  # noqa: E402

from mgcn import botnet  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devid", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--data_dir", default=None)
    ap.add_argument("--data_train", default="train.npz")
    ap.add_argument("--data_val", default="val.npz")
    ap.add_argument("--data_test", default="test.npz")
    ap.add_argument("--synthetic_nodes", type=int, default=143_107)
    ap.add_argument("--bsz", type=int, default=1)
    ap.add_argument("--shuffle", type=int, default=0)
    ap.add_argument("--enc_sizes", type=int, nargs="*", default=[32] * 8)
    ap.add_argument("--act", default="relu")
    ap.add_argument("--layer_act", default="relu")
    ap.add_argument("--residual_hop", type=int, default=0)
    ap.add_argument("--final", default="proj", choices=["none", "proj"])
    ap.add_argument("--deg_norm", default="sm", choices=["None", "sm", "rw"])
    ap.add_argument("--aggr", default="add", choices=["add", "mean", "max"])
    ap.add_argument("--dropout", type=float, default=0.0)
    ap.add_argument("--bias", type=int, default=0)
    ap.add_argument("--focal", action="store_true")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--weight_decay", type=float, default=5e-4)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--save_path", default=None)
    args = ap.parse_args()
    torch.manual_seed(args.seed)
    if args.data_dir:
        ds = [botnet.GraphDataset(os.path.join(args.data_dir, f))
              for f in (args.data_train, args.data_val, args.data_test)]
    else:
        tmp = tempfile.mkdtemp()
        ds = []
        for i, name in enumerate(("train", "val", "test")):
            path = os.path.join(tmp, f"{name}.npz")
            botnet.save_npz(botnet.synthetic_botnet(2 if name == "train" else 1, seed=10 * i,
                                                    n_nodes=args.synthetic_nodes), path)
            ds.append(botnet.GraphDataset(path))
    hist = botnet.train(*ds, enc_sizes=args.enc_sizes, residual_hop=args.residual_hop,
                        deg_norm=None if args.deg_norm == "None" else args.deg_norm,
                        aggr=args.aggr, bias=args.bias, dropout=args.dropout, final=args.final,
                        act=args.act, layer_act=args.layer_act, lr=args.lr,
                        weight_decay=args.weight_decay, epochs=args.epochs, batch_size=args.bsz,
                        shuffle=bool(args.shuffle), focal=args.focal,
                        device=f"cuda:{args.devid}", save_path=args.save_path,
                        log=lambda s: print(s, file=sys.stderr))
    print(json.dumps({"workload": "config3 botnet training (train_botnet.py)",
                      "data": args.data_dir or "synthetic", **hist}))


if __name__ == "__main__":
    main()
