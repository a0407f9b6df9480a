"""MPNN Q-network (src/networks/mpnn.py) on the HIP engine.

`MPNN` keeps the reference's module/parameter names and shapes, so reference
state_dicts (`network_best_*.pth`, dqn.py:604-610) load unchanged.  All parameters
are views into ONE flat fp32 buffer in state_dict order (58,425 floats for
n_obs_in=7): the optimiser and the multi-GPU gradient all-reduce work on that
flat buffer.  torch holds the memory; the forward is libecohip's fused kernel.
"""
import ctypes

import numpy as np
import torch

from .. import _lib
from ..graphs import GraphStore, dense_to_csr

N_FEATURES = 64


def param_layout(n_obs_in=7):
    """(name, shape) in state_dict order (mpnn.py:20-32, 86-87, 111-112, 129-139)."""
    lay = [("node_init_embedding_layer.0.weight", (64, n_obs_in)),
           ("edge_embedding_layer.edge_embedding_NN.weight", (63, n_obs_in + 1)),
           ("edge_embedding_layer.edge_feature_NN.weight", (64, 64))]
    for i in range(3):
        lay.append((f"update_node_embedding_layer.{i}.message_layer.weight", (64, 128)))
        lay.append((f"update_node_embedding_layer.{i}.update_layer.weight", (64, 128)))
    lay += [("readout_layer.layer_pooled.weight", (64, 64)),
            ("readout_layer.layers_readout.0.weight", (1, 128)),
            ("readout_layer.layers_readout.0.bias", (1,))]
    return lay


class MPNN(torch.nn.Module):
    """MPNN(n_obs_in, n_layers=3, n_features=64, tied_weights=False, n_hid_readout=[])."""

    def __init__(self, n_obs_in=7, n_layers=3, n_features=64, tied_weights=False, n_hid_readout=[],
                 device=None):
        super().__init__()
        if n_layers != 3 or n_features != N_FEATURES or tied_weights or list(n_hid_readout):
            raise NotImplementedError("eco_hip implements the ECO-DQN MPNN configuration used by the "
                                      "reference (n_layers=3, n_features=64, untied, no hidden readout)")
        if not 1 <= n_obs_in <= _lib.ECO_MPNN_MAX_OBS:
            raise ValueError("n_obs_in must be in [1, 16]")
        self.n_obs_in = n_obs_in
        self.n_layers = n_layers
        self.n_features = n_features
        dev = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        n = _lib.lib.eco_mpnn_param_count(n_obs_in)
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self._names = []
        off = 0
        for name, shape in param_layout(n_obs_in):
            cnt = int(np.prod(shape))
            p = torch.nn.Parameter(self.flat[off:off + cnt].view(shape))
            self._names.append(name)
            self._register_dotted(name, p)
            off += cnt
        assert off == n
        self.packed = torch.zeros(_lib.lib.eco_mpnn_packed_count(), dtype=torch.float32, device=dev)
        self._packed_version = -1
        self._ws = None
        self.timer = None   # optional list: (start_event, end_event, batch, n_spins) per forward launch

    def _register_dotted(self, name, p):
        """Register `p` under its exact reference state_dict key (nested submodules)."""
        parts = name.split(".")
        mod = self
        for part in parts[:-1]:
            if part not in mod._modules:
                mod.add_module(part, torch.nn.Module())
            mod = mod._modules[part]
        mod.register_parameter(parts[-1], p)

    # ---- parameters ----
    def flat_params(self):
        return self.flat

    def repack(self, stream=None):
        _lib.check(_lib.lib.eco_mpnn_pack(_lib.ptr(self.flat), self.n_obs_in, _lib.ptr(self.packed),
                                          _lib.stream_ptr(stream)))
        self._packed_version = self.flat._version

    def _ensure_packed(self, stream=None):
        if self._packed_version != self.flat._version:
            self.repack(stream)

    def load_state_dict(self, state_dict, strict=True):
        with torch.no_grad():
            for name, p in zip(self._names, self.parameters()):
                p.copy_(torch.as_tensor(state_dict[name]).to(p.device, p.dtype).view(p.shape))
        self._packed_version = -1

    def init_normal_(self, std, generator=None):
        """dqn.py:199-205: Linear weights ~ normal(0, std); biases keep their init."""
        with torch.no_grad():
            for name, p in zip(self._names, self.parameters()):
                if name.endswith("weight"):
                    p.copy_(torch.randn(p.shape, generator=generator) * std)
                else:
                    bound = 1.0 / np.sqrt(128)
                    p.copy_((torch.rand(p.shape, generator=generator) * 2 - 1) * bound)
        self._packed_version = -1

    def _check_x(self, obs_x):
        w = _lib.obs_x_stride(self.n_obs_in)
        if obs_x.dim() != 3 or obs_x.shape[2] != w or not obs_x.is_contiguous() or obs_x.dtype != torch.float32:
            raise ValueError(f"obs_x must be a contiguous float32 [B, N, {w}] tensor for n_obs_in={self.n_obs_in}")

    def _workspace(self, n_spins, batch):
        need = _lib.lib.eco_mpnn_workspace_bytes(n_spins, batch)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.flat.device)
        return self._ws

    # ---- fast path: graphs resident in a GraphStore ----
    def forward_graphs(self, obs_x, graphs, graph_ids, norm_scope=_lib.ECO_NORM_PER_GRAPH, q_out=None,
                       act=None, actions_out=None, saved=None, stream=None):
        """Q [B, N] for node features obs_x [B, N, W] (W = 8, or 16 for n_obs_in > 8) on graphs graph_ids [B].
        act: optional ActConfig -> fused epsilon-greedy actions written to actions_out [B] int32.
        saved: optional buffer (saved_bytes) that receives the activations for backward()."""
        B, N = obs_x.shape[0], obs_x.shape[1]
        self._check_x(obs_x)
        self._ensure_packed(stream)
        if q_out is None and act is None:
            q_out = torch.empty(B, N, dtype=torch.float32, device=obs_x.device)
        gids = graph_ids if graph_ids.dtype == torch.int32 else graph_ids.to(torch.int32)
        if self.timer is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        _lib.check(_lib.lib.eco_mpnn_forward(
            _lib.ptr(self.packed), self.n_obs_in, ctypes.byref(graphs.gs), _lib.ptr(gids.contiguous()), B,
            _lib.ptr(obs_x), norm_scope, _lib.ptr(q_out), ctypes.byref(act) if act is not None else None,
            _lib.ptr(actions_out), _lib.ptr(saved), _lib.ptr(self._workspace(N, B)), _lib.stream_ptr(stream)))
        if self.timer is not None:
            ev[1].record()
            self.timer.append((ev[0], ev[1], B, graph_ids))
        return q_out

    def forward_pair_graphs(self, other, obs_x, graphs, graph_ids, norm_scope=_lib.ECO_NORM_PER_GRAPH, q_out=None,
                            act=None, actions_out=None, q_out_other=None, act_other=None, actions_out_other=None,
                            stream=None):
        """This network and `other` on the same graphs and node features (the double-DQN pair of
        dqn.py:416-428: online argmax and target Q on s') -- eco_mpnn_forward_pair: one launch for one-graph
        dense blocks, else two forwards.  Returns (q_out, q_out_other)."""
        B, N = obs_x.shape[0], obs_x.shape[1]
        self._check_x(obs_x)
        if other.n_obs_in != self.n_obs_in:
            raise ValueError("paired networks must take the same observables")
        self._ensure_packed(stream)
        other._ensure_packed(stream)
        if q_out is None and act is None:
            q_out = torch.empty(B, N, dtype=torch.float32, device=obs_x.device)
        if q_out_other is None and act_other is None:
            q_out_other = torch.empty(B, N, dtype=torch.float32, device=obs_x.device)
        gids = graph_ids if graph_ids.dtype == torch.int32 else graph_ids.to(torch.int32)
        if self.timer is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        _lib.check(_lib.lib.eco_mpnn_forward_pair(
            _lib.ptr(self.packed), _lib.ptr(other.packed), self.n_obs_in, ctypes.byref(graphs.gs),
            _lib.ptr(gids.contiguous()), B, _lib.ptr(obs_x), norm_scope, _lib.ptr(q_out),
            ctypes.byref(act) if act is not None else None, _lib.ptr(actions_out), _lib.ptr(q_out_other),
            ctypes.byref(act_other) if act_other is not None else None, _lib.ptr(actions_out_other),
            _lib.ptr(self._workspace(N, B)), _lib.stream_ptr(stream)))
        if self.timer is not None:
            ev[1].record()
            self.timer.append((ev[0], ev[1], 2 * B, graph_ids))  # two forwards' work
        return q_out, q_out_other

    @staticmethod
    def saved_bytes(n_spins, batch):
        return _lib.lib.eco_mpnn_saved_bytes(n_spins, batch)

    def backward_graphs(self, obs_x, graphs, graph_ids, saved, dq, grad_out, workspace=None, stream=None):
        """loss.backward(): grad_out[flat] = dLoss/dparams for dq = dLoss/dQ [B, N] of the forward that
        filled `saved` (forward_graphs(..., norm_scope=ECO_NORM_PER_CALL, saved=...))."""
        B, N = obs_x.shape[0], obs_x.shape[1]
        self._check_x(obs_x)
        need = _lib.lib.eco_mpnn_backward_workspace_bytes(N, B)
        if workspace is None or workspace.numel() < need:
            workspace = torch.empty(need, dtype=torch.uint8, device=obs_x.device)
        gids = graph_ids if graph_ids.dtype == torch.int32 else graph_ids.to(torch.int32)
        if self.timer is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        _lib.check(_lib.lib.eco_mpnn_backward(
            _lib.ptr(self.packed), self.n_obs_in, ctypes.byref(graphs.gs), _lib.ptr(gids.contiguous()), B,
            _lib.ptr(obs_x), _lib.ptr(saved), _lib.ptr(dq), _lib.ptr(grad_out), _lib.ptr(workspace),
            _lib.stream_ptr(stream)))
        if self.timer is not None:
            ev[1].record()
            self.timer.append((ev[0], ev[1], -B, graph_ids))   # negative batch marks a backward launch
        return grad_out

    # ---- reference-format forward (drop-in for mpnn.py:40-77) ----
    def forward(self, obs):
        """obs [B, n_obs_in+N, N] or [n_obs_in+N, N] -> Q [B, N] (squeezed like mpnn.py:75).
        Reproduces the in-place transpose_ of a 3-D input (mpnn.py:44) and the batch-wide
        norm.max() (mpnn.py:102).  The dense adjacency rows are converted to CSR on the
        host: this path is for API compatibility; batched callers use forward_graphs."""
        if obs.dim() == 2:
            view = obs.unsqueeze(0)
        else:
            view = obs
        B, R, N = view.shape
        k = self.n_obs_in
        x = torch.zeros(B, N, _lib.obs_x_stride(k), dtype=torch.float32, device=self.flat.device)
        x[:, :, :k] = view[:, :k, :].transpose(1, 2).to(x.device, torch.float32)
        adj = view[:, k:, :].detach().cpu().numpy()
        store = GraphStore(*dense_to_csr([a.T for a in adj]), device=self.flat.device)
        gids = torch.arange(B, dtype=torch.int32, device=self.flat.device)
        q = self.forward_graphs(x, store, gids, norm_scope=_lib.ECO_NORM_PER_CALL)
        if obs.dim() == 3:
            obs.transpose_(-1, -2)   # mpnn.py:44 mutates the caller's tensor
        return q.squeeze()
