"""Config 1 on the GPU: the kernel/ model families on mgcn convs and the
10-fold CV driver run end to end on a MUTAG-shaped
synthetic dataset.  Accuracy values are not pinned (the TU data are absent
and PyG is not importable): the checks are the protocol (six results,
shapes, log-probabilities) and that a model learns."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

NETS = ["GCN", "GCNWithJK", "GraphSAGE", "GraphSAGEWithJK", "GIN0", "GIN0WithJK", "GIN",
        "GINWithJK"]


@pytest.mark.parametrize("net", NETS)
def test_models_forward_backward(cuda, net):
    import mgcn.kernel as K
    torch.manual_seed(0)
    ds = K.synthetic_tu(n_graphs=40)
    model = getattr(K, net)(ds, 3, 32).to(cuda)
    model.reset_parameters()
    batch = K.Batch.from_data_list([ds[i] for i in range(16)]).to(cuda)
    out = model(batch)
    assert out.shape == (16, 2)
    torch.testing.assert_close(out.exp().sum(1), torch.ones(16, device=cuda))
    torch.nn.functional.nll_loss(out, batch.y).backward()
    grads = [p.grad for p in model.parameters() if p.requires_grad]
    assert all(g is not None and torch.isfinite(g).all() for g in grads)


def test_cross_validation_protocol(cuda):
    import mgcn.kernel as K
    torch.manual_seed(0)
    ds = K.synthetic_tu()
    res = K.cross_validation_with_val_set(ds, K.GCN(ds, 2, 32), folds=4, epochs=3,
                                          batch_size=32, lr=0.01, lr_decay_factor=0.5,
                                          lr_decay_step_size=2, weight_decay=0, device=cuda,
                                          logger=None)
    assert len(res) == 6 and all(math.isfinite(v) for v in res)
    assert 0.0 <= res[1] <= 1.0 and 0.0 <= res[4] <= 1.0


def test_gcn_learns_synthetic_mutag(cuda):
    import mgcn.kernel as K
    torch.manual_seed(0)
    ds = K.synthetic_tu()
    model = K.GCN(ds, 2, 32).to(cuda)
    model.reset_parameters()
    opt = torch.optim.Adam(model.parameters(), lr=0.01)
    loader = K.DataLoader(ds, 32, shuffle=True)
    for _ in range(30):
        K.train_eval.train(model, opt, loader, cuda)
    acc = K.train_eval.eval_acc(model, K.DataLoader(ds, 64), cuda)
    assert acc > 0.8, acc
