"""Config-1 surface of the reference's kernel/ benchmark (TU graph
classification, 10-fold CV): offline TU loader + PyG-style batching
(``data``), the cross-validation driver (``train_eval``) and the
GCN / GraphSAGE / GIN model families on mgcn's convs (``models``)."""
from .data import (Batch, Data, DataLoader, NodeFeatureOnes, NormalizedDegree, OneHotDegree,
                   TUDataset, get_dataset, read_tu_data, synthetic_tu)
from .models import (GCN, GIN, GIN0, GCNWithJK, GIN0WithJK, GINWithJK, GraphSAGE,
                     GraphSAGEWithJK)
from .train_eval import (EarlyStopping, cross_validation_with_val_set, k_fold, run_sweep)

__all__ = ["Batch", "Data", "DataLoader", "NodeFeatureOnes", "NormalizedDegree", "OneHotDegree",
           "TUDataset", "get_dataset", "read_tu_data", "synthetic_tu", "GCN", "GCNWithJK",
           "GraphSAGE", "GraphSAGEWithJK", "GIN0", "GIN0WithJK", "GIN", "GINWithJK",
           "EarlyStopping", "cross_validation_with_val_set", "k_fold", "run_sweep"]
