"""Convert a botnet HDF5 dataset (the reference's layout: file attribute
num_graphs; group str(i) per graph with datasets x, y, edge_index, edge_y and
attributes num_nodes, ...) into mgcn.botnet's .npz layout.  Needs h5py, which
this image does not have: run it where the data and h5py live.

    python scripts/botnet_h5_to_npz.py chord_no100k_ev10k_us_train.hdf5 train.npz
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meta-gcn_amd")]


def main(src, dst):
    import h5py
    from mgcn.botnet import save_npz
    graphs = []
    with h5py.File(src, "r") as f:
        for i in range(int(f.attrs["num_graphs"])):
            grp = f[str(i)]
            g = {k: v[()] for k, v in grp.items()}
            g.update(dict(grp.attrs.items()))
            graphs.append(g)
    save_npz(graphs, dst)
    print(f"{src}: {len(graphs)} graphs -> {dst}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
