"""Transformer encoder text classifier (reference ``transformer.py:12-371``).

Parameter names and shapes are identical to the reference so checkpoints interchange
(survey §2.8): ``input_embeddings.{token,pos,segment}_embedding``,
``sublayer_attention.i.multiheads.heads.{0,1,2}``, ``...multiheads.output``,
``...layernorm.{a_2,b_2}``, ``sublayer_ffn.i.ffn.w_{1,2}``, ``pooler.dense``,
``classifier.classifier.{W1,b1,W2,b2}`` (2-D biases).

Model-defining quirks that are preserved: the embedding is added twice
(``x = emb + dropout(emb + pe)``, ``transformer.py:62-64``, Q14), pre-LN residuals with
no final LayerNorm, LayerNorm with *unbiased* std and eps added to std
(``transformer.py:239-242``), ``sqrt(d_model)`` embedding scale, tanh pooler on token 0,
manifold mixup of the pooled vector (``transformer.py:71-80``).

Bugs fixed by default, reproducible with ``faithful=True`` (survey §2.9):
Q7 attention mask fill ``-1e-9`` (no masking) -> real masking; Q8 manifold mixup active
in eval -> disabled in eval; Q5 FusedMLP bias grads averaged (1/B) -> summed.

On MI355X the hot ops dispatch to HIP kernels (``ops/layernorm.py``,
``ops/attention.py``, ``ops/embedding.py``, ``ops/mlp.py``).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import ffn
from ..ops.dropout import dropout_add, gelu_dropout
from ..ops.attention import packed_attention, scaled_dot_product_attention
from ..ops.embedding import embedding_sum
from ..ops.layernorm import ResidualGrad, layer_norm_unbiased
from ..ops.linear import linear, linear_cat
from ..ops.mlp import fused_mlp


class Transformer(nn.Module):
    def __init__(self, n_class, vocab, n_layers=6, h=8, d_model=512, d_ff=1024, d_hidden=1024,
                 maxlen=512, dropout_encodings=0.1, dropout_connection_attention=0.1,
                 dropout_connection_ffn=0.1, dropout_attention=0.1, dropout_ffn=0.1,
                 alpha=0.99, faithful=False):
        super().__init__()
        self.input_embeddings = Embeddings(d_model, vocab, maxlen)
        self.input_encodings = PositionalEncoding(d_model, dropout_encodings, maxlen)
        self.sublayer_attention = nn.ModuleList()
        self.sublayer_ffn = nn.ModuleList()
        for _ in range(n_layers):
            self.sublayer_attention.append(sublayerConnectionAttention(
                h, d_model, dropout_attention, dropout_connection_attention, faithful))
            self.sublayer_ffn.append(sublayerConnectionFFN(d_model, d_ff, dropout_ffn, dropout_connection_ffn))
        self.pooler = Pooler(d_model)
        self.dropout_post = nn.Dropout(0.1)
        self.classifier = Classifier(d_model, d_hidden, n_class, faithful)
        self.n_layers = n_layers
        self.alpha = alpha
        self.faithful = faithful
        # (perm, lam[B]) device tensors that replace the in-forward sampling (a HIP-graph
        # runner samples outside the captured region and writes them before each replay)
        self.mix_override = None
        self.init_params()

    def flat_adjacent(self, scope="shape"):
        """Parameter groups the flat buffers keep adjacent, in this order (utils/flat.py).
        ``scope`` "shape": all parameters of one shape, in registration order.  Then (1) each
        attention block's Q / K / V weights and biases sit back to back, so the fused projection
        reads the stacked bf16 weights as one view of the shadow buffer (no per-forward
        concatenation), and (2) NGD's batched shape groups are views of the flat gradient (no
        stack / scatter copies, optim/ngd.py ``_group_view``).  ``scope`` "layer": (1) only --
        each block's own Q / K / V (weights, biases), so the gradient buckets of a data-parallel
        run keep following the backward's layer order."""
        if scope == "layer":
            out = []
            for m in self.modules():
                heads = getattr(m, "heads", None)
                if isinstance(heads, nn.ModuleList) and len(heads) > 1 and all(isinstance(h, nn.Linear) for h in heads):
                    for attr in ("weight", "bias"):
                        grp = [getattr(h, attr) for h in heads]
                        if all(p is not None and p.requires_grad for p in grp):
                            out.append(grp)
            return out
        by_shape = {}
        for p in self.parameters():
            if p.requires_grad:
                by_shape.setdefault(tuple(p.shape), []).append(p)
        return [g for g in by_shape.values() if len(g) > 1]

    def sample_lam(self) -> float:
        """The manifold-mixup coefficient (host sample, as the reference's ``.item()``)."""
        if self.alpha > 0:
            return float(torch.distributions.beta.Beta(self.alpha, self.alpha).sample())
        return float(self.alpha)

    def forward(self, x, token_types, index, mask=None):
        """Returns ``(logits, perm_index, lam)`` like the reference (``transformer.py:84``).
        ``mask`` is the ``(B,1,1,L)`` attention mask (1 = keep)."""
        embeddings = self.input_embeddings(x, token_types, index)
        encodings = self.input_encodings(embeddings)
        x = embeddings + encodings
        if mask is not None:
            mask = mask.reshape(mask.shape[0], mask.shape[-1])
            if mask.dtype != torch.uint8:
                # once per forward, not once per layer (the attention kernels take uint8)
                mask = (mask != 0).to(torch.uint8)
        for i in range(self.n_layers):
            x = self.sublayer_attention[i](x, mask)
            x = self.sublayer_ffn[i](x)
        x = self.pooler(x)
        x = self.dropout_post(x)
        b = x.size(0)
        mix = self.training or self.faithful
        if mix and self.mix_override is not None:
            from ..ops.mixup import mixup_interpolate
            perm, lam_t = self.mix_override
            return self.classifier(mixup_interpolate(x, perm, lam_t)), perm, lam_t
        lam = self.sample_lam() if mix else 1.0
        if mix:
            perm = torch.randperm(b, device=x.device)
            from ..ops.mixup import mixup_interpolate
            cls = mixup_interpolate(x, perm, lam)
        else:
            perm = torch.arange(b, device=x.device)
            cls = x
        return self.classifier(cls), perm, lam

    def init_params(self, default_initialization=False):
        if not default_initialization:
            for _, p in self.named_parameters():
                if p.dim() > 1:
                    nn.init.xavier_uniform_(p)


class Pooler(nn.Module):
    def __init__(self, hidden_size):
        super().__init__()
        self.dense = nn.Linear(hidden_size, hidden_size)

    def forward(self, x):
        return torch.tanh(self.dense(x[:, 0, :]))


class PositionalEncoding(nn.Module):
    """Sinusoidal table, deliberately *not* a buffer (absent from the state_dict, like
    ``transformer.py:121``)."""

    def __init__(self, d_model, dropout, max_len):
        super().__init__()
        self.dropout = nn.Dropout(p=dropout)
        pe = torch.zeros(max_len, d_model)
        position = torch.arange(0, max_len).unsqueeze(1).float()
        scale = torch.exp(torch.arange(0, d_model, 2).float() * -(math.log(10000.0) / d_model))
        pe[:, 0::2] = torch.sin(position * scale)
        pe[:, 1::2] = torch.cos(position * scale)
        self.pe = pe.unsqueeze(0)
        self._pe_cache = {}

    def table(self, device, dtype):
        key = (device, dtype)
        t = self._pe_cache.get(key)
        if t is None:
            t = self.pe.to(device=device, dtype=dtype)
            self._pe_cache[key] = t
        return t

    def forward(self, x):
        return self.dropout(x + self.table(x.device, x.dtype)[:, :x.size(1)])


class Embeddings(nn.Module):
    """token + learned position + segment embedding, times sqrt(d_model)
    (``transformer.py:132-156``).  The token gather runs in fp32 like the reference
    (autocast disabled there)."""

    def __init__(self, d_model, vocab, maxlen):
        super().__init__()
        self.token_embedding = nn.Embedding(vocab, d_model)
        self.pos_embedding = nn.Embedding(maxlen, d_model)
        self.segment_embedding = nn.Embedding(3, d_model)
        self.d_model = d_model
        self.maxlen = maxlen

    def forward(self, x, token_types, index):
        L = x.size(1)
        pos_ids = index[:L] if index is not None else torch.arange(L, device=x.device)
        return embedding_sum(x, token_types, pos_ids, self.token_embedding.weight,
                             self.pos_embedding.weight, self.segment_embedding.weight,
                             math.sqrt(self.d_model))


class PositionalWiseFFN(nn.Module):
    def __init__(self, d_model, d_ff, dropout=0.1):
        super().__init__()
        self.w_1 = nn.Linear(d_model, d_ff)
        self.w_2 = nn.Linear(d_ff, d_model)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x, fuse_out_bias=False):
        """``fuse_out_bias``: the caller's dropout_add computes w_2's bias gradient (ops/dropout.py
        ``bias=``); w_1's is always computed inside the GELU-dropout backward.  On the GPU the
        w_1 GEMM carries the bias + GELU + dropout epilogue and w_2's data gradient the
        GELU-dropout backward (ops/ffn.py)."""
        if ffn.fusable(x, self.w_1.in_features, self.w_1.out_features):
            return ffn.ffn_core(x, self.w_1.weight, self.w_1.bias, self.w_2.weight, self.w_2.bias, self.dropout.p,
                                self.training, out_bias_grad=not fuse_out_bias)
        h = gelu_dropout(linear(x, self.w_1.weight, self.w_1.bias, bias_grad=False), self.dropout.p, self.training,
                         bias=self.w_1.bias)
        return linear(h, self.w_2.weight, self.w_2.bias, bias_grad=not fuse_out_bias)


class MultiheadAttention(nn.Module):
    """Q/K/V as three separate ``Linear`` (``heads.{0,1,2}``) + ``output``
    (``transformer.py:196-227``).  Unlike the reference the probabilities are not kept
    (``self.attn``): the fused kernel never materialises them."""

    def __init__(self, h, d_model, dropout=0.1, faithful=False):
        super().__init__()
        assert d_model % h == 0
        self.d_k = d_model // h
        self.h = h
        self.heads = nn.ModuleList([nn.Linear(d_model, d_model) for _ in range(3)])
        self.output = nn.Linear(d_model, d_model)
        self.dropout = nn.Dropout(p=dropout)
        self.faithful = faithful
        self.attn = None

    def forward(self, query, key, value, mask=None, fuse_out_bias=False):
        """``fuse_out_bias``: the caller's dropout_add computes the output projection's bias
        gradient (ops/dropout.py ``bias=``)."""
        b, L, _ = query.shape
        if query is key and key is value:
            qkv = linear_cat(query, [l.weight for l in self.heads], [l.bias for l in self.heads])
            qkv = qkv.view(b, L, 3, self.h, self.d_k)
            p = self.dropout.p if self.training else 0.0
            x = packed_attention(qkv, mask, dropout_p=p, mask_value=(-1e-9 if self.faithful else None))
            return linear(x.reshape(b, L, self.h * self.d_k), self.output.weight, self.output.bias,
                          bias_grad=not fuse_out_bias)
        q, k, v = [l(t).view(b, -1, self.h, self.d_k) for l, t in zip(self.heads, (query, key, value))]
        p = self.dropout.p if self.training else 0.0
        x = scaled_dot_product_attention(q, k, v, mask, dropout_p=p,
                                         mask_value=(-1e-9 if self.faithful else None))
        return linear(x.reshape(b, L, self.h * self.d_k), self.output.weight, self.output.bias,
                      bias_grad=not fuse_out_bias)


class LayerNorm(nn.Module):
    """``a_2 * (x - mean) / (std_unbiased + eps) + b_2`` (``transformer.py:230-242``)."""

    def __init__(self, features, eps=1e-6):
        super().__init__()
        self.a_2 = nn.Parameter(torch.ones(features))
        self.b_2 = nn.Parameter(torch.zeros(features))
        self.eps = eps

    def forward(self, x, res=None):
        return layer_norm_unbiased(x, self.a_2, self.b_2, self.eps, res=res)


class sublayerConnectionAttention(nn.Module):  # noqa: N801 (reference name)
    def __init__(self, h, d_model, dropout_head=0.1, dropout_connection=0.1, faithful=False):
        super().__init__()
        self.multiheads = MultiheadAttention(h, d_model, dropout_head, faithful)
        self.layernorm = LayerNorm(d_model)
        self.dropout = nn.Dropout(p=dropout_connection)

    def forward(self, x, mask=None):
        res = ResidualGrad()  # skip gradient handed to the LayerNorm backward (no add pass)
        y = self.layernorm(x, res)
        y = self.multiheads(y, y, y, mask, fuse_out_bias=True)
        return dropout_add(y, x, self.dropout.p, self.training, res, bias=self.multiheads.output.bias)


class sublayerConnectionFFN(nn.Module):  # noqa: N801 (reference name)
    def __init__(self, d_model, d_ff, dropout_ffn=0.1, dropout_connection=0.1):
        super().__init__()
        self.ffn = PositionalWiseFFN(d_model, d_ff, dropout_ffn)
        self.layernorm = LayerNorm(d_model)
        self.dropout = nn.Dropout(p=dropout_connection)

    def forward(self, x):
        res = ResidualGrad()
        y = self.ffn(self.layernorm(x, res), fuse_out_bias=True)
        return dropout_add(y, x, self.dropout.p, self.training, res, bias=self.ffn.w_2.bias)


class Classifier(nn.Module):
    def __init__(self, d_model, d_hidden, n_class, faithful=False):
        super().__init__()
        self.classifier = FusedMLP(d_model, d_hidden, n_class, faithful=faithful)

    def forward(self, x):
        return self.classifier(x)


class FusedMLP(nn.Module):
    """Linear -> ReLU -> Linear with 2-D biases ``(1, hidden)``/``(1, out)``
    (``transformer.py:341-371``).  ``faithful=True`` reproduces the reference's
    bias-gradient averaging (Q5)."""

    def __init__(self, input_channel, hidden_channel, output_channel, bias=True, device=None,
                 dtype=None, faithful=False):
        super().__init__()
        fk = {"device": device, "dtype": dtype}
        self.W1 = nn.Parameter(torch.empty(hidden_channel, input_channel, **fk))
        self.b1 = nn.Parameter(torch.empty(1, hidden_channel, **fk)) if bias else None
        self.W2 = nn.Parameter(torch.empty(output_channel, hidden_channel, **fk))
        self.b2 = nn.Parameter(torch.empty(1, output_channel, **fk)) if bias else None
        self.faithful = faithful
        self.reset_parameters()

    def forward(self, X):
        return fused_mlp(X, self.W1, self.b1, self.W2, self.b2, bias_grad_mean=self.faithful)

    def reset_parameters(self):
        nn.init.xavier_uniform_(self.W1)
        nn.init.xavier_uniform_(self.W2)
        if self.b1 is not None:
            nn.init.constant_(self.b1, 0.0)
        if self.b2 is not None:
            nn.init.constant_(self.b2, 0.0)
