"""AG News text pipeline (reference ``transformer_test.py:59-149``, survey D6).

Reference behaviour: torchtext ``AG_NEWS`` datapipes -> per-batch collate that strips HTML
(``<...>``) and URLs, removes gensim stopwords, tokenises with ``bert-base-uncased``
(``padding='longest'``, no truncation -> Q18) and returns
``(input_ids, labels 1..4, token_type_ids, attention_mask)``; labels are shifted by -1 in
the training loop; vocab = 30522.

MI355X design:

* the whole corpus is tokenised ONCE up front (not per batch in worker processes) into a
  packed int32 token store ``(offsets, tokens)`` with per-sample lengths; a batch is a
  gather + pad on the device (static shapes per length bucket);
* sequences are truncated to ``max_len`` (512, the model's position table; fixes Q18);
* ``length_buckets`` (e.g. 64/128/256/512) round each batch's padded length up so the
  attention/GEMM shapes repeat (kernel tuning and HIP-graph friendly); ``None`` pads to
  the longest sample in the batch exactly like the reference;
* tokenizer: the HuggingFace tokenizer the reference uses (``bert-base-uncased``, from the
  local HF cache or a directory path).  If it cannot be loaded the run FAILS; the
  dependency-free ``HashWordPieceTokenizer`` (lower-casing word tokenizer hashing words into
  the BERT id range with BERT's special ids [PAD]=0, [CLS]=101, [SEP]=102) is used only when
  asked for by name (``--tokenizer hash``);
* data: the AG News CSVs (``train.csv``/``test.csv``, rows ``"class","title","description"``,
  the files torchtext's ``AG_NEWS`` reads) under ``root/ag_news``, downloaded with MD5 checks
  (``AGNEWS_URLS`` / ``AGNEWS_MD5``) when missing.  A run that asks for real data and cannot
  get it raises; ``synthetic_agnews`` (an AG-News-shaped corpus: 120k/7.6k samples, 4
  classes, AG-News-like lengths, class-dependent vocabulary) is used only with
  ``synthetic=True`` (``--synthetic``);
* the tokenised corpus is cached next to the CSV (``tokens_<tokenizer>_<max_len>.npz``,
  keyed by the CSV's MD5), so later runs skip tokenisation.
"""
from __future__ import annotations

import csv
import hashlib
import os
import re
import zlib

import numpy as np
import torch

VOCAB_SIZE = 30522
PAD_ID, CLS_ID, SEP_ID = 0, 101, 102
NUM_CLASSES = 4
TRAIN_SIZE, TEST_SIZE = 120000, 7600

# the reference's cleaning regexes (transformer_test.py:73-79): tags removed without a
# separator, www-style URLs replaced by one space
_HTML = re.compile(r"<.*?>")
_URL = re.compile(r"\s*(?:https?://)?www\.\S*\.[A-Za-z]{2,5}\s*")

# The AG News CSVs (Zhang et al. 2015, as distributed with the char-CNN data and read by
# torchtext's AG_NEWS dataset, which the reference uses: transformer_test.py:88-93).
AGNEWS_URLS = {
    "train": "https://raw.githubusercontent.com/mhjabreel/CharCnn_Keras/master/data/ag_news_csv/train.csv",
    "test": "https://raw.githubusercontent.com/mhjabreel/CharCnn_Keras/master/data/ag_news_csv/test.csv",
}
AGNEWS_MD5 = {"train": "b1a00f826fdfbd249f79597b59e1dc12", "test": "d52ea96a97a2d943681189a97654912d"}
_WORD = re.compile(r"[a-z0-9]+(?:'[a-z]+)?|[^\sa-z0-9]")

# gensim.parsing.preprocessing.STOPWORDS (gensim 3.x/4.x), the list the reference's
# ``remove_stopwords`` uses (/root/reference/transformer_test.py:52,95): the 318-word Glasgow list
# (= scikit-learn's ENGLISH_STOP_WORDS) plus 19 additions (computer, did, didn, does, doesn, doing,
# don, just, kg, km, make, quite, really, regarding, say, unless, used, using, various) -- 337 words.
# gensim is not installed here; the constant is in-tree so the token stream matches the reference.
STOPWORDS = frozenset("""a about above across after afterwards again against all almost alone along already also although always am
among amongst amoungst amount an and another any anyhow anyone anything anyway anywhere are around as at back
be became because become becomes becoming been before beforehand behind being below beside besides between
beyond bill both bottom but by call can cannot cant co computer con could couldnt cry de describe detail did
didn do does doesn doing don done down due during each eg eight either eleven else elsewhere empty enough etc
even ever every everyone everything everywhere except few fifteen fifty fill find fire first five for former
formerly forty found four from front full further get give go had has hasnt have he hence her here hereafter
hereby herein hereupon hers herself him himself his how however hundred i ie if in inc indeed interest into is
it its itself just keep kg km last latter latterly least less ltd made make many may me meanwhile might mill
mine more moreover most mostly move much must my myself name namely neither never nevertheless next nine no
nobody none noone nor not nothing now nowhere of off often on once one only onto or other others otherwise our
ours ourselves out over own part per perhaps please put quite rather re really regarding same say see seem
seemed seeming seems serious several she should show side since sincere six sixty so some somehow someone
something sometime sometimes somewhere still such system take ten than that the their them themselves then
thence there thereafter thereby therefore therein thereupon these they thick thin third this those though
three through throughout thru thus to together too top toward towards twelve twenty two un under unless until
up upon us used using various very via was we well were what whatever when whence whenever where whereafter
whereas whereby wherein whereupon wherever whether which while whither who whoever whole whom whose why will
with within without would yet you your yours yourself yourselves""".split())
assert len(STOPWORDS) == 337
CLEAN_VERSION = "g337"  # cache tag of the cleaning rules (changes invalidate cached token stores)


def clean_text(s: str) -> str:
    """HTML strip + URL strip + stopword removal (reference ``transformer_test.py:73-79``,
    applied per sample in ``generate_batch``)."""
    s = _HTML.sub("", s)
    s = _URL.sub(" ", s).strip()
    # gensim's remove_stopwords: whitespace split, CASE-SENSITIVE membership ("The" stays)
    return " ".join(w for w in s.split() if w not in STOPWORDS)


class HashWordPieceTokenizer:
    """Deterministic offline tokenizer with BERT's id conventions."""

    vocab_size = VOCAB_SIZE
    first_regular = 1000  # BERT's [unused]/special block lives below
    name = "hash"

    def _id(self, w: str) -> int:
        return self.first_regular + zlib.crc32(w.encode()) % (VOCAB_SIZE - self.first_regular)

    def encode(self, text: str, max_len: int = 512):
        ids = [CLS_ID] + [self._id(w) for w in _WORD.findall(text.lower())]
        ids = ids[: max_len - 1] + [SEP_ID]
        return ids


class TokenizerUnavailable(RuntimeError):
    pass


def get_tokenizer(name_or_path: str | None = "bert-base-uncased"):
    """The named HF tokenizer (local cache or a directory; no network), or the hash
    tokenizer when ``name_or_path`` is ``"hash"``.  Raises ``TokenizerUnavailable`` when the
    named tokenizer cannot be loaded -- never substitutes another one silently."""
    if name_or_path in (None, "", "hash"):
        if name_or_path != "hash":
            raise TokenizerUnavailable("no tokenizer named (use 'bert-base-uncased', a path, or 'hash')")
        return HashWordPieceTokenizer()
    os.environ.setdefault("HF_HUB_OFFLINE", "1")
    try:
        from transformers import AutoTokenizer
        tok = AutoTokenizer.from_pretrained(name_or_path, local_files_only=True)
    except Exception as e:  # noqa: BLE001 - any loader failure is reported as one error
        raise TokenizerUnavailable(
            f"tokenizer {name_or_path!r} cannot be loaded offline ({type(e).__name__}: {e}); put it in the HF cache "
            f"or pass a directory, or pass --tokenizer hash to use the built-in hash tokenizer explicitly") from e

    class _HF:
        vocab_size = tok.vocab_size
        name = str(name_or_path)

        def encode(self, text, max_len=512):
            return tok(text, truncation=True, max_length=max_len)["input_ids"]

        def encode_batch(self, texts, max_len=512):
            return tok(list(texts), truncation=True, max_length=max_len)["input_ids"]
    return _HF()


def get_tokenizer_size(name_or_path: str | None = "bert-base-uncased") -> int:
    """Reference ``get_tokenizer_size`` (``transformer_test.py:141-143``)."""
    return get_tokenizer(name_or_path).vocab_size


class TokenStore:
    """Packed corpus: ``tokens`` (int32, concatenated), ``offsets`` [n+1], ``labels`` [n]
    (0-based)."""

    def __init__(self, seqs, labels):
        lens = np.fromiter((len(s) for s in seqs), dtype=np.int64, count=len(seqs))
        self.offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        self.tokens = np.fromiter((t for s in seqs for t in s), dtype=np.int32, count=int(lens.sum()))
        self.labels = np.asarray(labels, dtype=np.int64)
        self.lengths = lens

    def __len__(self):
        return len(self.labels)

    def sample(self, i):
        return self.tokens[self.offsets[i]:self.offsets[i + 1]], int(self.labels[i])


def read_agnews_csv(path: str):
    """AG News CSV rows ``"class","title","description"`` -> (texts, 0-based labels); the
    text is the row's fields after the class joined by a space (torchtext's AG_NEWS)."""
    texts, labels = [], []
    with open(path, newline="", encoding="utf-8") as f:
        for row in csv.reader(f):
            if len(row) < 2:
                continue
            labels.append(int(row[0]) - 1)  # reference shifts labels by -1 (transformer_test.py:242)
            texts.append(clean_text(" ".join(row[1:])))
    return texts, labels


def synthetic_agnews(n: int, seed: int = 0, max_len: int = 512, vocab: int = VOCAB_SIZE):
    """AG-News-shaped corpus: lengths ~ the BERT-tokenised AG News distribution (mean ~45,
    long tail to ~200), 4 balanced classes, each with a class-specific vocabulary slice
    mixed into shared background tokens so a model can learn it."""
    rng = np.random.default_rng(seed)
    lens = np.clip(np.rint(rng.lognormal(mean=3.75, sigma=0.33, size=n)), 8, max_len - 2).astype(np.int64)
    labels = rng.integers(0, NUM_CLASSES, size=n)
    span = (vocab - 1000) // (NUM_CLASSES + 1)
    seqs = []
    for L, c in zip(lens, labels):
        bg = rng.integers(1000, 1000 + span, size=L)
        topic = rng.integers(1000 + span * (c + 1), 1000 + span * (c + 2), size=L)
        pick = rng.random(L) < 0.3
        body = np.where(pick, topic, bg)
        seqs.append(np.concatenate([[CLS_ID], body, [SEP_ID]]).astype(np.int32))
    return TokenStore(seqs, labels)


def agnews_csv(root: str, split: str) -> str:
    return os.path.join(root, "ag_news", f"{split}.csv")


def download_agnews(root: str = "./data", splits=("train", "test")) -> list[str]:
    """Fetch the AG News CSVs into ``root/ag_news`` (skipped when present with the right
    MD5; a corrupted or truncated file is fetched again).  Call on one rank, then barrier."""
    from .download import download_url
    out = []
    for sp in splits:
        out.append(download_url(AGNEWS_URLS[sp], os.path.join(root, "ag_news"), f"{sp}.csv", AGNEWS_MD5[sp]))
    return out


def _tokenize_cached(path: str, tok, max_len: int) -> TokenStore:
    with open(path, "rb") as fh:
        digest = hashlib.md5(fh.read(), usedforsecurity=False).hexdigest()
    name = re.sub(r"[^A-Za-z0-9_.-]+", "_", getattr(tok, "name", type(tok).__name__))
    cache = os.path.join(os.path.dirname(path), f"tokens_{os.path.basename(path)[:-4]}_{name}_{max_len}_{CLEAN_VERSION}.npz")
    if os.path.isfile(cache):
        z = np.load(cache)  # (allow_pickle=False: plain arrays only)
        if str(z["md5"]) == digest:
            st = TokenStore.__new__(TokenStore)
            st.offsets, st.tokens, st.labels = z["offsets"], z["tokens"], z["labels"]
            st.lengths = np.diff(st.offsets)
            return st
    texts, labels = read_agnews_csv(path)
    if hasattr(tok, "encode_batch"):
        seqs = []
        for i in range(0, len(texts), 4096):
            seqs.extend(tok.encode_batch(texts[i:i + 4096], max_len))
    else:
        seqs = [tok.encode(t, max_len) for t in texts]
    st = TokenStore(seqs, labels)
    try:
        tmp = cache + ".tmp.npz"
        np.savez(tmp, offsets=st.offsets, tokens=st.tokens, labels=st.labels, md5=np.array(digest))
        os.replace(tmp, cache)
    except OSError:
        pass  # read-only data directory: no cache
    return st


def load_agnews(root: str = "./data", train: bool = True, tokenizer=None, max_len: int = 512,
                synthetic: bool = False, seed: int = 0, download: bool = True):
    """TokenStore for the split.  ``synthetic``: the AG-News-shaped synthetic corpus.
    Otherwise the real CSV under ``root/ag_news`` -- downloaded first when missing and
    ``download`` -- tokenised with ``tokenizer``; raises ``FileNotFoundError`` when the data
    cannot be had (no silent substitute)."""
    if synthetic:
        return synthetic_agnews(TRAIN_SIZE if train else TEST_SIZE, seed=seed + (0 if train else 1),
                                max_len=max_len)
    split = "train" if train else "test"
    path = agnews_csv(root, split)
    if not os.path.isfile(path) and download:
        try:
            download_agnews(root, (split,))
        except Exception as e:  # noqa: BLE001
            raise FileNotFoundError(f"AG News {split} split not found at {path} and the download failed "
                                    f"({type(e).__name__}: {e}); place the CSV there or pass --synthetic") from e
    if not os.path.isfile(path):
        raise FileNotFoundError(f"AG News {split} split not found at {path} (download disabled); "
                                f"place the CSV there or pass --synthetic")
    if tokenizer is None:
        raise TokenizerUnavailable("load_agnews: real data needs a tokenizer (get_tokenizer(...))")
    return _tokenize_cached(path, tokenizer, max_len)


def _round_up(L, buckets):
    if not buckets:
        return L
    for b in buckets:
        if L <= b:
            return b
    return buckets[-1]


class TextBatchLoader:
    """Batches of ``(input_ids [B,L], labels [B], token_type_ids [B,L], attention_mask [B,L])``
    with DistributedSampler semantics (seeded shared permutation, rank-strided shard,
    ``set_epoch``, ``drop_last``).

    ``resident`` (default): the packed token store is uploaded to the device once and a
    batch is one device gather + pad; only the batch's sample indices and lengths cross
    the bus.  ``resident=False`` (corpora larger than wanted in HBM, e.g. a real CSV of
    any size): the host gathers + pads the token ids and stages them.  On a GPU every
    per-batch transfer goes through the pinned ring + copy stream of ``prefetch.py``
    (staged one batch ahead, no pageable copy, no host sync)."""

    def __init__(self, store: TokenStore, batch_size: int, device, rank=0, world_size=1, shuffle=True,
                 drop_last=True, seed=0, length_buckets=(64, 128, 256, 512), resident=True, pinned=None):
        self.store = store
        self.bs = batch_size
        self.device = torch.device(device)
        self.rank, self.world = rank, world_size
        self.shuffle, self.drop_last, self.seed = shuffle, drop_last, seed
        self.buckets = sorted(length_buckets) if length_buckets else None
        self.epoch = 0
        self.resident = resident
        if pinned is None:
            pinned = self.device.type == "cuda"
        self.stager = None
        if pinned:
            from .prefetch import PinnedStager
            lmax = int(store.lengths.max()) if len(store) else 1
            if self.buckets:
                lmax = _round_up(lmax, self.buckets)
            per = 2 * 8 * batch_size + 512 if resident else (4 * batch_size * lmax + 3 * 4 * batch_size + 1024)
            self.stager = PinnedStager(self.device, per, 3)
        if resident:
            self.tokens = torch.from_numpy(store.tokens.astype(np.int64)).to(self.device)
            self.offsets = torch.from_numpy(store.offsets).to(self.device)
            self.labels = torch.from_numpy(store.labels).to(self.device)
        self._types = {}

    def set_epoch(self, e):
        self.epoch = e

    def _indices(self):
        n = len(self.store)
        perm = (torch.randperm(n, generator=torch.Generator().manual_seed(self.seed + self.epoch))
                if self.shuffle else torch.arange(n))
        per = n // self.world if self.drop_last else -(-n // self.world)
        if not self.drop_last and per * self.world > n:
            perm = torch.cat([perm, perm[: per * self.world - n]])
        return perm[self.rank:per * self.world:self.world]

    def __len__(self):
        per = len(self.store) // self.world if self.drop_last else -(-len(self.store) // self.world)
        return per // self.bs if self.drop_last else -(-per // self.bs)

    # ---- host half: what crosses the bus for one batch
    def _host(self, idx: np.ndarray):
        lens = self.store.lengths[idx]
        L = _round_up(int(lens.max()), self.buckets)
        ln = np.minimum(lens, L).astype(np.int64)
        if self.resident:
            return [idx.astype(np.int64), ln], L
        B = idx.size
        starts = self.store.offsets[idx]
        pos = np.arange(L)
        valid = pos[None, :] < ln[:, None]
        gat = np.minimum(starts[:, None] + pos[None, :], max(len(self.store.tokens) - 1, 0))
        ids = np.where(valid, self.store.tokens[gat], PAD_ID).astype(np.int32)
        return [ids.reshape(B, L), self.store.labels[idx].astype(np.int32), ln], L

    # ---- device half: build the batch from the transferred tensors
    def _device(self, arrs, L):
        pos = torch.arange(L, device=self.device)
        if self.resident:
            dev_idx, ln = arrs
            start = self.offsets[dev_idx]
            valid = pos.unsqueeze(0) < ln.unsqueeze(1)
            gather = (start.unsqueeze(1) + pos.unsqueeze(0)).clamp(max=self.tokens.numel() - 1)
            ids = torch.where(valid, self.tokens[gather], torch.zeros((), dtype=torch.long, device=self.device))
            labels = self.labels[dev_idx]
        else:
            ids32, lab32, ln = arrs
            valid = pos.unsqueeze(0) < ln.unsqueeze(1)
            ids = ids32.long()
            labels = lab32.long()
        B = ids.shape[0]
        types = self._types.get((B, L))
        if types is None:
            types = self._types[(B, L)] = torch.zeros(B, L, dtype=torch.long, device=self.device)
        return ids, labels, types, valid.to(torch.long)

    def batch(self, idx):
        """One batch from sample indices (host tensor/array), without staging (CPU path)."""
        arrs, L = self._host(np.asarray(idx, dtype=np.int64))
        return self._device([torch.from_numpy(a).to(self.device) for a in arrs], L)

    def __iter__(self):
        idx = self._indices().numpy()
        nb = len(self)
        if self.stager is None:
            for b in range(nb):
                yield self.batch(idx[b * self.bs:(b + 1) * self.bs])
            return
        from .prefetch import StagedIterator
        yield from StagedIterator(self.stager, nb, lambda b: self._host(idx[b * self.bs:(b + 1) * self.bs]),
                                  self._device)
