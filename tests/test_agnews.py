"""AG News acquisition without silent substitutes (VERDICT r3 missing #2): download through
data/download.py with MD5 checks (file:// fixture), clean -> tokenize -> TokenStore, a
tokenised-corpus cache, and hard failures when the data or the named tokenizer is missing.
Reference: transformer_test.py:73-104 (AG_NEWS + cleaning + bert-base-uncased), :141-149."""
import csv
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

from faster_distributed_training_amd.data import agnews as A

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ROWS = [
    ("3", "Wall St. Bears Claw Back", "<p>Reuters - Short-sellers are seeing green again.</p>"),
    ("4", "New chip from the lab", "Visit www.example.com for the details of the new design"),
    ("2", "Team wins the final", "The home side won the cup after extra time"),
    ("1", "Talks resume", "Leaders of both nations met on Monday"),
] * 6


def _write_csv(d, name, rows):
    os.makedirs(d, exist_ok=True)
    p = os.path.join(d, name)
    with open(p, "w", newline="", encoding="utf-8") as f:
        csv.writer(f, quoting=csv.QUOTE_ALL).writerows(rows)
    with open(p, "rb") as f:
        return p, hashlib.md5(f.read()).hexdigest()


@pytest.fixture
def mirror(tmp_path, monkeypatch):
    """A file:// mirror of the two CSVs, with the module's URL / MD5 constants pointed at it."""
    src = tmp_path / "mirror"
    tr, md5_tr = _write_csv(str(src), "train.csv", ROWS)
    te, md5_te = _write_csv(str(src), "test.csv", ROWS[:8])
    monkeypatch.setattr(A, "AGNEWS_URLS", {"train": "file://" + tr, "test": "file://" + te})
    monkeypatch.setattr(A, "AGNEWS_MD5", {"train": md5_tr, "test": md5_te})
    return tmp_path / "data"


def test_clean_text_matches_reference_rules():
    s = A.clean_text("<b>Stocks</b> rise in the www.example.com market")
    assert "<" not in s and "www" not in s
    assert s.split() == ["Stocks", "rise", "market"]  # stopwords "in", "the" removed


def test_stopwords_are_gensims():
    """gensim's STOPWORDS (337 words) = scikit-learn's Glasgow list + 19 additions; gensim's
    remove_stopwords is case-sensitive (reference transformer_test.py:52,95)."""
    assert len(A.STOPWORDS) == 337
    try:
        from sklearn.feature_extraction.text import ENGLISH_STOP_WORDS
    except ImportError:
        ENGLISH_STOP_WORDS = None
    if ENGLISH_STOP_WORDS is not None:
        assert set(ENGLISH_STOP_WORDS) <= A.STOPWORDS
        assert sorted(A.STOPWORDS - set(ENGLISH_STOP_WORDS)) == sorted(
            "computer did didn does doesn doing don just kg km make quite really regarding say unless used using "
            "various".split())
    assert A.clean_text("The computer using km rose") == "The rose"


def test_download_clean_tokenize_store(mirror):
    tok = A.get_tokenizer("hash")
    st = A.load_agnews(str(mirror), True, tok, max_len=64)
    assert os.path.isfile(A.agnews_csv(str(mirror), "train"))  # downloaded into root/ag_news
    assert len(st) == len(ROWS)
    assert sorted(set(st.labels.tolist())) == [0, 1, 2, 3]  # 1..4 shifted to 0-based
    ids, lab = st.sample(0)
    assert ids[0] == A.CLS_ID and ids[-1] == A.SEP_ID and lab == 2
    # cleaning happened before tokenisation: same ids as the cleaned text
    assert list(ids) == tok.encode(A.clean_text(ROWS[0][1] + " " + ROWS[0][2]), 64)
    te = A.load_agnews(str(mirror), False, tok, max_len=64)
    assert len(te) == 8


def test_tokenised_corpus_cache(mirror, monkeypatch):
    tok = A.get_tokenizer("hash")
    st = A.load_agnews(str(mirror), True, tok, max_len=64)
    caches = [f for f in os.listdir(os.path.join(str(mirror), "ag_news")) if f.endswith(".npz")]
    assert len(caches) == 1 and "hash" in caches[0]
    monkeypatch.setattr(A, "read_agnews_csv", lambda p: (_ for _ in ()).throw(AssertionError("re-tokenised")))
    st2 = A.load_agnews(str(mirror), True, tok, max_len=64)
    assert np.array_equal(st.tokens, st2.tokens) and np.array_equal(st.offsets, st2.offsets)
    assert np.array_equal(st.labels, st2.labels) and np.array_equal(st.lengths, st2.lengths)


def test_md5_mismatch_is_an_error(mirror, monkeypatch):
    monkeypatch.setattr(A, "AGNEWS_MD5", {"train": "0" * 32, "test": "0" * 32})
    with pytest.raises(FileNotFoundError, match="download failed"):
        A.load_agnews(str(mirror), True, A.get_tokenizer("hash"))


def test_missing_data_raises(tmp_path, monkeypatch):
    monkeypatch.setattr(A, "AGNEWS_URLS", {"train": "file:///nonexistent/train.csv",
                                           "test": "file:///nonexistent/test.csv"})
    with pytest.raises(FileNotFoundError, match="--synthetic"):
        A.load_agnews(str(tmp_path), True, A.get_tokenizer("hash"))
    with pytest.raises(FileNotFoundError, match="download disabled"):
        A.load_agnews(str(tmp_path), True, A.get_tokenizer("hash"), download=False)
    # the synthetic corpus only when asked for
    assert len(A.load_agnews(str(tmp_path), True, None, synthetic=True)) == A.TRAIN_SIZE


def test_missing_tokenizer_raises(tmp_path):
    with pytest.raises(A.TokenizerUnavailable, match="--tokenizer hash"):
        A.get_tokenizer(str(tmp_path / "no_such_tokenizer"))
    with pytest.raises(A.TokenizerUnavailable):
        A.get_tokenizer(None)
    assert isinstance(A.get_tokenizer("hash"), A.HashWordPieceTokenizer)


def test_local_hf_tokenizer_directory(tmp_path, mirror):
    """The HF path (what bert-base-uncased takes from the cache) with a small local WordPiece
    tokenizer saved to a directory."""
    from transformers import BertTokenizer
    words = ["[PAD]"] + [f"[unused{i}]" for i in range(99)] + ["[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    words += sorted({w.lower() for r in ROWS for w in A.clean_text(r[1] + " " + r[2]).replace(".", " ").split()})
    BertTokenizer(vocab={w: i for i, w in enumerate(words)}, do_lower_case=True).save_pretrained(str(tmp_path / "tok"))
    tok = A.get_tokenizer(str(tmp_path / "tok"))
    assert tok.vocab_size == len(words)
    st = A.load_agnews(str(mirror), True, tok, max_len=32)
    ids, _ = st.sample(2)
    assert ids[0] == 101 and ids[-1] == 102 and len(ids) > 4  # [CLS] ... [SEP]


def _cli(args, cwd):
    env = dict(os.environ, FDT_NATIVE="0", PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, os.path.join(ROOT, "transformer_test.py")] + args, cwd=cwd, env=env,
                          capture_output=True, text=True, timeout=600)


def test_cli_without_data_fails(tmp_path):
    """No --synthetic, no CSV, no network: the reference-compatible CLI exits non-zero instead
    of training on fabricated data."""
    r = _cli(["-b", "4", "--epoch", "1", "--steps", "1", "--layers", "1", "--d_model", "32", "--no_plot",
              "--tokenizer", "hash", "--data_root", str(tmp_path / "empty")], tmp_path)
    assert r.returncode != 0
    assert "AG News" in (r.stdout + r.stderr) and "--synthetic" in (r.stdout + r.stderr)


def test_cli_trains_on_real_csv(tmp_path):
    d = tmp_path / "data" / "ag_news"
    _write_csv(str(d), "train.csv", ROWS)
    _write_csv(str(d), "test.csv", ROWS[:8])
    r = _cli(["-b", "4", "--epoch", "1", "--steps", "2", "--eval_steps", "1", "--layers", "1", "--d_model", "32",
              "--no_plot", "--tokenizer", "hash", "--data_root", str(tmp_path / "data")], tmp_path)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "epoch 0:" in r.stdout
    r = _cli(["-b", "4", "--epoch", "1", "--steps", "1", "--layers", "1", "--d_model", "32", "--no_plot",
              "--data_root", str(tmp_path / "data")], tmp_path)  # default bert-base-uncased: not cached here
    assert r.returncode != 0 and "--tokenizer hash" in (r.stdout + r.stderr)
