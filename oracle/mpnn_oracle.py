"""fp32 torch restatement of the reference MPNN Q-network and DQN train step
(TEST INFRASTRUCTURE ONLY -- the parity checker for the HIP kernels, never shipped).

Follows src/networks/mpnn.py line by line:
  MPNN.forward               :40-77   (in-place transpose_ at :44 is NOT reproduced
                                       here; the product wrapper reproduces it)
  get_normalisation          :34-38   (deg = #nonzero, clamped 0 -> 1)
  EdgeAndNodeEmbeddingLayer  :79-104  (norm.max() over the WHOLE batch at :102)
  UpdateNodeEmbeddingLayer   :106-120
  ReadoutLayer               :123-159
and src/agents/dqn/dqn.py:403-451 (train_step: double DQN, MSE, Adam).

Weights are a dict keyed by the reference state_dict names.
Pinned against the reference: tests/golden/mpnn_fwd.npz, dqn_step.npz.
"""
import torch
import torch.nn.functional as F

KEYS = [
    "node_init_embedding_layer.0.weight",            # [64, 7]
    "edge_embedding_layer.edge_embedding_NN.weight",  # [63, 8]
    "edge_embedding_layer.edge_feature_NN.weight",    # [64, 64]
    "update_node_embedding_layer.0.message_layer.weight",
    "update_node_embedding_layer.0.update_layer.weight",
    "update_node_embedding_layer.1.message_layer.weight",
    "update_node_embedding_layer.1.update_layer.weight",
    "update_node_embedding_layer.2.message_layer.weight",
    "update_node_embedding_layer.2.update_layer.weight",
    "readout_layer.layer_pooled.weight",              # [64, 64]
    "readout_layer.layers_readout.0.weight",          # [1, 128]
    "readout_layer.layers_readout.0.bias",            # [1]
]
SHAPES = [(64, 7), (63, 8), (64, 64)] + [(64, 128)] * 6 + [(64, 64), (1, 128), (1,)]
N_PARAMS = sum(int(torch.tensor(s).prod()) for s in SHAPES)   # 58,425


def shapes(n_obs_in=7):
    """Parameter shapes of MPNN(n_obs_in) in state_dict order (mpnn.py:20-23, :86-87, :111-112, :129-139)."""
    return [(64, n_obs_in), (63, n_obs_in + 1)] + SHAPES[2:]


def init_weights(gen, std=0.01, n_obs_in=7):
    """dqn.py:199-205: Linear weights ~ normal(0, std); the readout bias keeps its
    nn.Linear default U(-1/sqrt(128), 1/sqrt(128))."""
    w = {}
    for k, s in zip(KEYS, shapes(n_obs_in)):
        if k.endswith("bias"):
            w[k] = (torch.rand(s, generator=gen) * 2 - 1) / (128 ** 0.5)
        else:
            w[k] = torch.randn(s, generator=gen) * std
    return w


def forward(w, obs, n_obs_in=7, norm_max=None):
    """MPNN.forward on obs [B, n_obs_in+N, N] (or [n_obs_in+N, N]) -> Q [B, N] (squeezed like :75).
    norm_max: the `norm.max()` of mpnn.py:102, taken over the whole input tensor; pass the value of a
    larger batch explicitly to evaluate that batch in chunks (a chunk's own max would differ)."""
    if obs.dim() == 2:
        obs = obs.unsqueeze(0)
    obs = obs.transpose(-1, -2)                                       # :44 (copy, not in place)
    x = obs[:, :, 0:n_obs_in]
    adj = obs[:, :, n_obs_in:]
    norm = torch.sum((adj != 0), dim=1).unsqueeze(-1)                 # :36
    norm = norm.clone()
    norm[norm == 0] = 1                                               # :37
    norm = norm.float()
    h = F.relu(x @ w[KEYS[0]].T)                                      # :20-23, :55
    # EdgeAndNodeEmbeddingLayer (:89-104)
    B, N = adj.shape[0], adj.shape[1]
    ef = torch.cat([adj.unsqueeze(-1),
                    x.unsqueeze(-2).transpose(-2, -3).repeat(1, N, 1, 1)], dim=-1)
    ef = ef * (adj.unsqueeze(-1) != 0).float()
    emb = F.relu(ef.reshape(B, N * N, -1) @ w[KEYS[1]].T).reshape(B, N, N, -1)
    emb = emb.sum(dim=2) / norm
    nmax = norm.max() if norm_max is None else torch.as_tensor(float(norm_max), dtype=norm.dtype,
                                                                    device=norm.device)
    e = F.relu(torch.cat([emb, norm / nmax], dim=-1) @ w[KEYS[2]].T)
    for i in range(3):                                                # :68-72, :114-120
        agg = torch.matmul(adj, h) / norm
        m = F.relu(torch.cat([agg, e], dim=-1) @ w[KEYS[3 + 2 * i]].T)
        h = F.relu(torch.cat([h, m], dim=-1) @ w[KEYS[4 + 2 * i]].T)
    # ReadoutLayer (:143-159)
    pooled = (h.sum(dim=1) / N) @ w[KEYS[9]].T
    fp = pooled.unsqueeze(1).expand(B, N, pooled.shape[-1])
    feat = F.relu(torch.cat([fp, h], dim=-1))
    q = feat @ w[KEYS[10]].T + w[KEYS[11]]
    return q.squeeze()


def batch_norm_max(states, n_obs_in=7):
    """norm.max() of mpnn.py:102 for a whole batch of observations [B, n_obs_in+N, N]: the largest
    clamped nonzero count of an adjacency row (:36-37)."""
    return (states[:, n_obs_in:, :] != 0).sum(dim=2).clamp_min(1).max()


def forward_chunked(w, states, n_obs_in=7, chunk=None):
    """forward() of a batch evaluated `chunk` graphs at a time with the batch's own norm.max() (so the
    result is the whole batch's forward: the [k, N, N, 63] edge tensor of :90-100 stays bounded)."""
    if chunk is None or states.shape[0] <= chunk:
        return forward(w, states, n_obs_in).reshape(states.shape[0], -1)
    nmax = batch_norm_max(states, n_obs_in)
    return torch.cat([forward(w, states[i:i + chunk], n_obs_in, norm_max=nmax).reshape(-1, states.shape[-1])
                      for i in range(0, states.shape[0], chunk)])


def train_step(w, adam_state, states, actions, rewards, states_next, dones,
               gamma=0.95, lr=1e-4, eps=1e-8, target_w=None, double_dqn=True, n_obs_in=7,
               reversible=True, allowed_value=-1.0, chunk=None):
    """dqn.py:403-451.  Reversible env: gather/argmax over all N actions (:408-415).  Irreversible
    (S2V) env: actions whose spin row differs from the allowed action state are masked to -10000
    before the argmax / max (:417-428); a terminal s' (every action masked) gives argmax 0, and its
    (1 - done) factor zeroes the term.  `adam_state` = dict(step=int, m={k: tensor}, v={k: tensor});
    torch.optim.Adam semantics (bias-corrected, eps added to sqrt(v_hat)).  Returns (new_w, loss).
    chunk: evaluate the forwards and the loss gradient `chunk` graphs at a time (batch-global norm.max(),
    gradients accumulated over the chunks of the mean loss) to bound the oracle's memory."""
    target_w = w if target_w is None else target_w
    B = states_next.shape[0]
    with torch.no_grad():
        if reversible:
            if double_dqn:
                a_star = forward_chunked(w, states_next, n_obs_in, chunk).argmax(1, True)
                q_t = forward_chunked(target_w, states_next, n_obs_in, chunk).gather(1, a_star)
            else:
                q_t = forward_chunked(target_w, states_next, n_obs_in, chunk).max(1, True)[0]
        else:
            target_preds = forward_chunked(target_w, states_next, n_obs_in, chunk)
            disallowed = states_next[:, 0, :] != allowed_value
            if double_dqn:
                preds = forward_chunked(w, states_next, n_obs_in, chunk).masked_fill(disallowed, -10000)
                q_t = target_preds.gather(1, preds.argmax(1, True))
            else:
                q_t = target_preds.masked_fill(disallowed, -10000).max(1, True)[0]
    td = rewards + (1 - dones) * gamma * q_t
    wg = {k: v.clone().requires_grad_(True) for k, v in w.items()}
    if chunk is None or states.shape[0] <= chunk:
        q = forward(wg, states, n_obs_in).reshape(states.shape[0], -1).gather(1, actions)
        loss = F.mse_loss(q, td, reduction="mean")
        loss.backward()
    else:  # mean over B of the squared errors, one chunk's sum at a time
        nmax = batch_norm_max(states, n_obs_in)
        total = 0.0
        for i in range(0, B, chunk):
            q = forward(wg, states[i:i + chunk], n_obs_in, norm_max=nmax).reshape(-1, states.shape[-1])
            part = ((q.gather(1, actions[i:i + chunk]) - td[i:i + chunk]) ** 2).sum() / B
            part.backward()
            total += part.item()
        loss = torch.tensor(total)
    adam_state["grad"] = {k: wg[k].grad.detach().clone() for k in KEYS}  # loss.backward() result
    adam_state["step"] += 1
    t = adam_state["step"]
    new_w = {}
    with torch.no_grad():
        for k in KEYS:
            g = wg[k].grad
            m = adam_state["m"].setdefault(k, torch.zeros_like(g))
            v = adam_state["v"].setdefault(k, torch.zeros_like(g))
            m.mul_(0.9).add_(g, alpha=0.1)
            v.mul_(0.999).addcmul_(g, g, value=0.001)
            bc1 = 1 - 0.9 ** t
            bc2 = 1 - 0.999 ** t
            denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
            new_w[k] = w[k] - (lr / bc1) * m / denom
    return new_w, loss.item()
