"""gcn_meta module surface (src/gcn_meta/models/*) on the mgcn engine.

Same class names, constructor arguments, forward signatures, parameter names
and initialisation as the reference, so ``state_dict``s load in either
direction and the training scripts (src/run/train_botnet.py:190-294) run
unchanged after swapping the import:

  NodeModelBase / NodeModelAdditive  gcn_base_models.py:11-243
  GCNMultiKernel                     gcn_multi_kernel.py:9-114
  GCNLayer / GCNModel                gcn_model.py:8-197
  activation / Identity / scatter_   common.py:11-66

The aggregation (gather, degree normalisation, reduce, bias, ReLU) is one HIP
kernel per direction (:func:`mgcn.ops.aggregate`); the feature transform
``x @ W`` (gcn_base_models.py:201) runs on libmgcn's MFMA GEMMs through
:func:`mgcn.ops.linear` (bf16x6 arithmetic, fp32 accuracy), with a fused
backward (dW, dX, ReLU mask, bias column sums in one kernel); residual layers
fuse their skip projection into the same GEMM (:func:`mgcn.ops.residual_gcn_layer`).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
from torch.nn import Parameter
from torch.nn.utils.rnn import pad_sequence

from . import _lib as L
from .graph import plan_for
from .ops import (aggregate_plan, gcn_layer, gcn_stack, linear, linear_bias,  # noqa: F401
                  residual_gcn_layer, residual_layer_supported, residual_stack,  # noqa: F401
                  scatter_)


# --------------------------------------------------------------- inits (PyG)
def _wants_norm_grad(deg, edge_weight) -> bool:
    """A gradient is asked of deg / edge_weight (lists: the K kernels')."""
    if not torch.is_grad_enabled():
        return False
    ts = []
    for t in (deg, edge_weight):
        ts += list(t) if isinstance(t, (list, tuple)) else [t]
    return any(isinstance(t, torch.Tensor) and t.requires_grad for t in ts)


def glorot(tensor):
    """torch_geometric.nn.inits.glorot (used at gcn_base_models.py:193)."""
    if tensor is not None:
        stdv = math.sqrt(6.0 / (tensor.size(-2) + tensor.size(-1)))
        tensor.data.uniform_(-stdv, stdv)


def zeros(tensor):
    """torch_geometric.nn.inits.zeros (gcn_base_models.py:197)."""
    if tensor is not None:
        tensor.data.fill_(0)


class Linear(nn.Linear):
    """torch.nn.Linear with identical parameters/state_dict, whose products run
    on libmgcn (x W^T and dx on mgcn_gemm_nn, dW on the split-K mgcn_gemm_tn).
    Used for GCNModel's residual and final projections (gcn_model.py:64-73)."""

    def forward(self, input):
        return linear_bias(input, self.weight, self.bias)


# ------------------------------------------------------------- common.py
class Identity(nn.Module):
    """common.py:11-24"""

    def __init__(self, *args, **kwargs):
        super().__init__()

    def forward(self, input):
        return input


def activation(act, negative_slope=0.2):
    """common.py:27-34"""
    activations = nn.ModuleDict([
        ['lrelu', nn.LeakyReLU(negative_slope)],
        ['relu', nn.ReLU()],
        ['elu', nn.ELU()],
        ['none', Identity()],
    ])
    return activations[act]


# ------------------------------------------------------- gcn_base_models.py
class NodeModelBase(nn.Module):
    """gcn_base_models.py:11-160 (constructor checks and degnorm_const)."""

    def __init__(self, in_channels, out_channels, in_edgedim=None, deg_norm=None, edge_gate=None,
                 aggr='add', *args, **kwargs):
        assert deg_norm in [None, 'sm', 'rw']
        assert edge_gate in [None, 'proj', 'free']
        assert aggr in ['add', 'mean', 'max']
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.in_edgedim = in_edgedim
        self.deg_norm = deg_norm
        self.aggr = aggr
        if edge_gate is not None:
            # EdgeGateProj / EdgeGateFree (gcn_base_models.py:322-396) are
            # outside the aggregation hot path this engine accelerates.
            raise NotImplementedError(
                "edge_gate is not supported by the mgcn engine (not on the Â·X hot path)")
        self.register_parameter('edge_gate', None)

    @staticmethod
    def degnorm_const(edge_index=None, num_nodes=None, deg=None, edge_weight=None, method='sm',
                      device=None):
        """Normalisation constants exactly as gcn_base_models.py:65-146 returns
        them (size (E,), or (N,) for 'rw' without edge weights), computed by
        libmgcn (mgcn_degree_norm / mgcn_edge_norm) and returned in COO order;
        differentiable in edge_weight / deg when they require grad."""
        assert method in ['sm', 'rw']
        if edge_weight is None and deg is None:
            assert edge_index is not None and num_nodes is not None
        plan = plan_for(edge_index, int(num_nodes if num_nodes is not None else deg.numel()))
        norm = plan.norm(method, deg=deg, edge_weight=edge_weight)
        if method == 'rw' and edge_weight is None:
            return norm.dinv  # (with its autograd history when deg requires grad)
        eid = plan.fwd.eid.long()
        if norm.grad:
            return torch.zeros_like(norm.w_fwd).index_put((eid,), norm.w_fwd)
        out = torch.empty_like(norm.w_fwd)
        out[eid] = norm.w_fwd
        return out

    def forward(self, x, edge_index, edge_attr=None, deg=None, *args, **kwargs):
        return x

    def num_parameters(self):
        if not hasattr(self, 'num_para'):
            self.num_para = sum([p.nelement() for p in self.parameters()])
        return self.num_para

    def __repr__(self):
        return '{} (in_channels: {}, out_channels: {}, in_edgedim: {}, deg_norm: {}, edge_gate: {},' \
               'aggr: {} | number of parameters: {})'.format(
                   self.__class__.__name__, self.in_channels, self.out_channels, self.in_edgedim,
                   self.deg_norm, self.edge_gate.__class__.__name__, self.aggr,
                   self.num_parameters())


class NodeModelAdditive(NodeModelBase):
    """gcn_base_models.py:163-243: x @ W, normalised gather, reduce, + bias."""

    def __init__(self, in_channels, out_channels, in_edgedim=None, deg_norm='sm', edge_gate=None,
                 aggr='add', bias=True, **kwargs):
        super().__init__(in_channels, out_channels, in_edgedim, deg_norm, edge_gate, aggr,
                         **kwargs)
        self.weight_node = Parameter(torch.Tensor(in_channels, out_channels))
        if in_edgedim is not None:
            self.weight_edge = Parameter(torch.Tensor(in_edgedim, out_channels))
        if bias:
            self.bias = Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter('bias', None)
        self.reset_parameters()

    def reset_parameters(self):
        glorot(self.weight_node)
        if self.in_edgedim is not None:
            glorot(self.weight_edge)
        if self.bias is not None:
            zeros(self.bias)

    def forward(self, x, edge_index, edge_attr=None, deg=None, edge_weight=None, **kwargs):
        return self.forward_fused(x, edge_index, edge_attr, deg, edge_weight, relu=False)

    def forward_fused(self, x, edge_index, edge_attr=None, deg=None, edge_weight=None,
                      relu=False):
        """forward() with the caller's ReLU folded into the aggregation epilogue."""
        if edge_attr is not None:
            raise NotImplementedError(
                "edge_attr messages (gcn_base_models.py:204-227) are not supported by the "
                "mgcn engine")
        plan = plan_for(edge_index, x.size(0))
        # deg_norm None ignores edge_weight entirely (gcn_base_models.py:209-211)
        norm = plan.norm(self.deg_norm, deg=deg,
                         edge_weight=edge_weight if self.deg_norm is not None else None)
        if self.aggr != 'max':
            # torch.matmul(x, W) (gcn_base_models.py:201) fused behind the
            # aggregation where the kernels apply
            return gcn_layer(x, self.weight_node, plan, norm, self.aggr, self.bias, relu)
        x = linear(x, self.weight_node)  # torch.matmul(x, W), gcn_base_models.py:201
        return aggregate_plan(x, plan, norm, self.aggr, self.bias, relu)


# ------------------------------------------------------ gcn_multi_kernel.py
class GCNMultiKernel(nn.Module):
    """gcn_multi_kernel.py:9-114.  Only the 'additive' node model runs on this
    engine; attention / hard-attention node models are out of scope."""

    nodemodel_dict = {'additive': NodeModelAdditive}

    def __init__(self, *args, num_kernel=1, nodemodel='additive', kernel_combine='add',
                 **kwargs):
        assert nodemodel in ['additive', 'attention', 'hardattention']
        assert kernel_combine in ['add', 'cat', 'mean']
        super().__init__()
        if nodemodel != 'additive':
            raise NotImplementedError(f"nodemodel={nodemodel!r} is not supported by mgcn")
        self.kernel_combine = kernel_combine
        self.node_models = nn.ModuleList(
            [self.nodemodel_dict[nodemodel](*args, **kwargs) for k in range(num_kernel)])

    def reset_parameters(self):
        for net in self.node_models:
            net.reset_parameters()

    @staticmethod
    def _listify(edge_index_K, edge_attr_K, deg_K, edge_weight_K):
        # gcn_multi_kernel.py:77-91
        if isinstance(edge_index_K, torch.Tensor):
            edge_index_K = [edge_index_K]
        if isinstance(edge_attr_K, torch.Tensor):
            edge_attr_K = [edge_attr_K]
        if isinstance(deg_K, torch.Tensor):
            deg_K = [deg_K]
        if isinstance(edge_weight_K, torch.Tensor):
            edge_weight_K = [edge_weight_K]
        n = len(edge_index_K)
        return (edge_index_K, edge_attr_K or [None] * n, deg_K or [None] * n,
                edge_weight_K or [None] * n)

    def forward(self, x, edge_index_K, edge_attr_K=None, deg_K=None, edge_weight_K=None,
                **kwargs):
        return self.forward_fused(x, edge_index_K, edge_attr_K, deg_K, edge_weight_K, relu=False)

    def can_fuse_relu(self, edge_index_K) -> bool:
        if isinstance(edge_index_K, torch.Tensor):
            edge_index_K = [edge_index_K]
        return len(self.node_models) == 1 and len(edge_index_K) == 1 \
            and edge_index_K[0] is not None

    def forward_fused(self, x, edge_index_K, edge_attr_K=None, deg_K=None, edge_weight_K=None,
                      relu=False):
        eis, eas, degs, ews = self._listify(edge_index_K, edge_attr_K, deg_K, edge_weight_K)
        if relu:
            assert self.can_fuse_relu(edge_index_K)
            return self.node_models[0].forward_fused(x, eis[0], eas[0], degs[0], ews[0],
                                                     relu=True)
        xo = None
        outs = []
        for nm, edge_index, edge_attr, deg, edge_weight in zip(self.node_models, eis, eas, degs,
                                                               ews):
            if edge_index is None:
                continue
            y = nm(x, edge_index, edge_attr, deg, edge_weight)
            outs.append(y)
        if not outs:
            return 0
        if self.kernel_combine == 'cat':
            # the reference's `xo != 0` test breaks for K > 1 (gcn_multi_kernel.py:100);
            # the intended concatenation is done here
            return torch.cat(outs, dim=1)
        xo = outs[0]
        for y in outs[1:]:
            xo = xo + y
        if self.kernel_combine == 'mean':
            xo = xo / len(outs)
        return xo


# -------------------------------------------------------------- gcn_model.py
class GCNLayer(nn.Module):
    """gcn_model.py:128-197; a ReLU layer activation is fused into the
    aggregation epilogue when there is a single kernel."""

    def __init__(self, in_channels, out_channels, in_edgedim=None, deg_norm='sm', edge_gate=None,
                 aggr='add', bias=True, num_kernel=1, nodemodel='additive', non_linear='relu',
                 **kwargs):
        super().__init__()
        kwargs.pop('nheads', None)  # attention-only argument (gcn_model.py:49)
        self.gcn = GCNMultiKernel(in_channels, out_channels, in_edgedim, deg_norm=deg_norm,
                                  edge_gate=edge_gate, aggr=aggr, bias=bias,
                                  num_kernel=num_kernel, nodemodel=nodemodel, **kwargs)
        self.non_linear = activation(non_linear)
        self.non_linear_name = non_linear
        self._relu = non_linear == 'relu'

    def reset_parameters(self):
        self.gcn.reset_parameters()

    def forward(self, x, edge_index_K, edge_attr_K=None, deg_K=None, edge_weight_K=None,
                **kwargs):
        if self._relu and self.gcn.can_fuse_relu(edge_index_K):
            return self.gcn.forward_fused(x, edge_index_K, edge_attr_K, deg_K, edge_weight_K,
                                          relu=True)
        xo = self.gcn(x, edge_index_K, edge_attr_K, deg_K, edge_weight_K, **kwargs)
        return self.non_linear(xo)


class GCNStack(nn.Module):
    """A plain chain of GCNLayers (the config-2 model: 3 layers, ReLU between)
    executed as ONE fused autograd node (:func:`mgcn.ops.gcn_stack`) whenever
    every layer is a single additive kernel with the same deg_norm/aggr and a
    'relu'/'none' activation; otherwise layer by layer.  Parameters live in
    the GCNLayer modules (reference-compatible state_dict keys)."""

    def __init__(self, layers):
        super().__init__()
        self.layers = nn.ModuleList(layers)

    def _fusable(self):
        nms = []
        for layer in self.layers:
            g = layer.gcn
            if len(g.node_models) != 1 or layer.non_linear_name not in ('relu', 'none'):
                return None
            nms.append(g.node_models[0])
        if len({(nm.deg_norm, nm.aggr) for nm in nms}) != 1:
            return None
        return nms

    def forward(self, x, edge_index, deg=None, edge_weight=None):
        nms = self._fusable()
        if nms is None or x.device.type != "cuda":
            for layer in self.layers:
                x = layer(x, edge_index, None, deg, edge_weight)
            return x
        plan = plan_for(edge_index, x.size(0))
        norm = plan.norm(nms[0].deg_norm, deg=deg,
                         edge_weight=edge_weight if nms[0].deg_norm is not None else None)
        relus = [layer.non_linear_name == 'relu' for layer in self.layers]
        return gcn_stack(x, plan, norm, [nm.weight_node for nm in nms], [nm.bias for nm in nms],
                         relus, nms[0].aggr)


class GCNModel(nn.Module):
    """gcn_model.py:8-125: GCN layers, residual Linear every `residual_hop`
    layers, dropout, optional final projection, optional graph mean-pool."""

    def __init__(self, in_channels, enc_sizes, num_classes, non_linear='relu',
                 non_linear_layer_wise='relu', residual_hop=None, dropout=0.5,
                 final_layer_config=None, final_type='none', pred_on='node', **kwargs):
        assert final_type in ['none', 'proj']
        assert pred_on in ['node', 'graph']
        super().__init__()
        self.in_channels = in_channels
        self.enc_sizes = [in_channels, *enc_sizes]
        self.num_layers = len(self.enc_sizes) - 1
        self.num_classes = num_classes
        self.residual_hop = residual_hop
        self.non_linear_layer_wise = non_linear_layer_wise
        self.final_type = final_type
        self.pred_on = pred_on
        if 'nheads' in kwargs:
            if isinstance(kwargs['nheads'], int):
                self.nheads = [kwargs['nheads']] * self.num_layers
            elif isinstance(kwargs['nheads'], list):
                self.nheads = kwargs['nheads']
                assert len(self.nheads) == self.num_layers
            else:
                raise ValueError
            del kwargs['nheads']
        else:
            self.nheads = [1] * self.num_layers
        if final_layer_config is None:
            self.gcn_net = nn.ModuleList([
                GCNLayer(in_c, out_c, nheads=nh, non_linear=non_linear_layer_wise, **kwargs)
                for in_c, out_c, nh in zip(self.enc_sizes, self.enc_sizes[1:], self.nheads)])
        else:
            assert isinstance(final_layer_config, dict)
            self.gcn_net = nn.ModuleList([
                GCNLayer(in_c, out_c, nheads=nh, non_linear=non_linear_layer_wise, **kwargs)
                for in_c, out_c, nh in zip(self.enc_sizes[:-2], self.enc_sizes[1:-1],
                                           self.nheads[:-1])])
            kwargs.update(final_layer_config)
            self.gcn_net.append(GCNLayer(self.enc_sizes[-2], self.enc_sizes[-1],
                                         nheads=self.nheads[-1],
                                         non_linear=non_linear_layer_wise, **kwargs))
        self.dropout = nn.Dropout(dropout)
        if residual_hop is not None and residual_hop > 0:
            self.residuals = nn.ModuleList([
                Linear(self.enc_sizes[i], self.enc_sizes[j])
                for i, j in zip(range(0, len(self.enc_sizes), residual_hop),
                                range(residual_hop, len(self.enc_sizes), residual_hop))])
            self.non_linear = activation(non_linear)
            self.num_residuals = len(self.residuals)
        if self.final_type == 'none':
            self.final = nn.Identity()
        elif self.final_type == 'proj':
            self.final = Linear(self.enc_sizes[-1], num_classes)
        else:
            raise ValueError

    def reset_parameters(self):
        for net in self.gcn_net:
            net.reset_parameters()
        if self.residual_hop is not None:
            for net in self.residuals:
                net.reset_parameters()
        if self.final_type != 'none':
            self.final.reset_parameters()

    fuse_residual = True  # class switch (tests compare against the step-for-step path)

    def _residual_fusable(self, x, edge_index_K, edge_attr_K):
        """residual_hop = 1 with single additive kernels, ReLU joins and no
        active dropout: each layer + its residual runs as one fused node."""
        if not self.fuse_residual or self.residual_hop != 1 or \
                getattr(self, 'num_residuals', 0) != self.num_layers:
            return False
        if not isinstance(edge_index_K, torch.Tensor) or edge_attr_K is not None:
            return False
        if x.device.type != "cuda" or not isinstance(self.non_linear, nn.ReLU):
            return False
        if self.training and self.dropout.p > 0:
            return False
        for layer in self.gcn_net:
            if len(layer.gcn.node_models) != 1 or layer.non_linear_name not in ('relu', 'none'):
                return False
        return True

    def forward(self, x, edge_index_K, edge_attr_K=None, deg_K=None, edge_weight_K=None,
                **kwargs):
        if (self._residual_fusable(x, edge_index_K, edge_attr_K) and
                not _wants_norm_grad(deg_K, edge_weight_K)):
            x = self._forward_residual_fused(x, edge_index_K, deg_K, edge_weight_K)
            return self._readout(x, **kwargs)
        # gcn_model.py:86-125, step for step
        xr = None
        add_xr_at = -1
        for n, net in enumerate(self.gcn_net):
            xo = net(x, edge_index_K, edge_attr_K, deg_K, edge_weight_K, **kwargs)
            xo = self.dropout(xo)
            if self.residual_hop is not None and self.residual_hop > 0:
                if n % self.residual_hop == 0 and (n // self.residual_hop) < self.num_residuals:
                    xr = self.residuals[n // self.residual_hop](x)
                    add_xr_at = n + self.residual_hop - 1
                if n == add_xr_at:
                    if n < self.num_layers - 1:
                        xo = self.non_linear(xo + xr)
                    else:
                        xo = xo + xr
            x = xo
        return self._readout(x, **kwargs)

    def _forward_residual_fused(self, x, edge_index, deg, edge_weight):
        if isinstance(deg, (list, tuple)):
            deg = deg[0]
        if isinstance(edge_weight, (list, tuple)):
            edge_weight = edge_weight[0]
        plan = plan_for(edge_index, x.size(0))
        last = self.num_layers - 1
        items = []
        for n, (layer, res) in enumerate(zip(self.gcn_net, self.residuals)):
            nm = layer.gcn.node_models[0]
            norm = plan.norm(nm.deg_norm, deg=deg,
                             edge_weight=edge_weight if nm.deg_norm is not None else None)
            items.append((nm, norm, layer.non_linear_name == 'relu', n < last, res))
        n = 0
        while n < len(items):
            nm, norm, relu1, relu2, res = items[n]
            # a run of 32 -> 32 layers on the same normalisation and aggregator:
            # one fused stack node (one host call per direction)
            m = n
            while (m < len(items) and items[m][1] is norm and items[m][0].aggr == nm.aggr and
                   residual_layer_supported(plan, x, items[m][0].weight_node,
                                            items[m][4].weight, L.REDUCE_CODES[nm.aggr])):
                m += 1
            if m - n >= 2:
                x = residual_stack(x, plan, norm, nm.aggr, [it[2] for it in items[n:m]],
                                   [it[3] for it in items[n:m]],
                                   [(it[0].weight_node, it[0].bias, it[4].weight, it[4].bias)
                                    for it in items[n:m]])
                n = m
                continue
            x = residual_gcn_layer(x, plan, norm, nm.aggr, relu1, relu2, nm.weight_node, nm.bias,
                                   res.weight, res.bias)
            n += 1
        return x

    def _readout(self, x, **kwargs):
        x = self.final(x)
        if self.pred_on == 'graph':
            assert 'batch_slices_x' in kwargs
            batch_slices_x = kwargs['batch_slices_x']
            if len(batch_slices_x) == 2:
                x = x.mean(dim=0, keepdim=True)
            else:
                x_batch, lengths = zip(*[(x[i:j], j - i) for (i, j) in
                                         zip(batch_slices_x, batch_slices_x[1:])])
                x_batch = pad_sequence(x_batch, batch_first=True, padding_value=0)
                x = x_batch.sum(dim=1) / x_batch.new_tensor(lengths)
        return x


__all__ = ["glorot", "zeros", "Identity", "activation", "scatter_", "Linear", "NodeModelBase",
           "NodeModelAdditive", "GCNMultiKernel", "GCNLayer", "GCNStack", "GCNModel"]
_ = L  # keep the binding imported so a missing library fails at import of ops
