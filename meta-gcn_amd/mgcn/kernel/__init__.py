"""Config-1 surface of the reference's kernel/ benchmark (TU graph
classification, 10-fold CV): offline TU loader + PyG-style batching
(``data``), the cross-validation driver (``train_eval``) and the
GCN / GraphSAGE / GIN model families on mgcn's convs (``models``) and the
pooling-operator nets (``pool_nets``, on :mod:`mgcn.pool`)."""
from .data import (Batch, Data, DataLoader, DenseData, DenseDataLoader, NodeFeatureOnes,
                   NormalizedDegree, OneHotDegree, ToDense, TUDataset, get_dataset, read_tu_data,
                   synthetic_tu)
from .models import (GCN, GIN, GIN0, GCNWithJK, GIN0WithJK, GINWithJK, GraphSAGE,
                     GraphSAGEWithJK)
from .pool_nets import (NETS, DiffPool, EdgePool, GlobalAttentionNet, Graclus, HardPool,
                        SAGPool, SAGPoolNew, Set2SetNet, SortPool, TopK, TopKNew)
from .train_eval import (EarlyStopping, cross_validation_with_val_set, k_fold, run_sweep)

__all__ = ["DenseData", "DenseDataLoader", "ToDense", "NETS", "DiffPool", "EdgePool",
           "GlobalAttentionNet", "Graclus", "HardPool", "SAGPool", "SAGPoolNew", "Set2SetNet",
           "SortPool", "TopK", "TopKNew",
           "Batch", "Data", "DataLoader", "NodeFeatureOnes", "NormalizedDegree", "OneHotDegree",
           "TUDataset", "get_dataset", "read_tu_data", "synthetic_tu", "GCN", "GCNWithJK",
           "GraphSAGE", "GraphSAGEWithJK", "GIN0", "GIN0WithJK", "GIN", "GINWithJK",
           "EarlyStopping", "cross_validation_with_val_set", "k_fold", "run_sweep"]
