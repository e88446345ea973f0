"""Reference parity of the AWD-LSTM serving path: sampler rule, detokenizer, vocab I/O."""
import math
import pickle

import pytest
import torch

from hipzap.serve import text as T


def test_select_token_rule():
    # first draw that is neither 0 nor excluded, else the first draw (main.py:63-68)
    assert T.select_token([0, 5, 7], {5}) == 7
    assert T.select_token([0, 5, 0], {5}) == 0
    assert T.select_token([3, 4], set()) == 3


def test_detokenizer_rules():
    d = T.Detokenizer()
    d.add_prompt("")
    for w in ["hello", "world", ".", "this", "is", "n't", "it", "!", "yes", "'s", "\n", "ok"]:
        d.add(w)
    assert d.text == "  hello world. This isn't it! Yes's \n Ok"


def test_gumbel_topk_distribution_matches_softmax():
    torch.manual_seed(0)
    logits = torch.tensor([2.0, 1.0, 0.0, -1.0, 0.5])
    p = torch.softmax(logits, 0)
    g = torch.Generator().manual_seed(1)
    n = 20000
    counts = torch.zeros(5)
    for _ in range(n):
        counts[T.gumbel_topk(logits, 1, g)[0]] += 1
    chi2 = (((counts - n * p) ** 2) / (n * p)).sum().item()
    assert chi2 < 20.5  # 4 dof, p ~ 4e-4


def test_gumbel_topk_without_replacement_and_stable():
    logits = torch.tensor([1000.0, 999.0, -5.0, 3.0])  # exp() of these overflows fp32
    idx = T.gumbel_topk(logits, 4)
    assert sorted(idx.tolist()) == [0, 1, 2, 3]


def test_itos_loading_safe(tmp_path):
    itos = ["xxunk", "xxpad", "hello"]
    p = tmp_path / "v.itos.pkl"
    T.save_itos(itos, str(p))
    assert T.load_itos(str(p)) == itos
    j = tmp_path / "v.json"
    T.save_itos(itos, str(j))
    assert T.load_itos(str(j)) == itos

    class Evil:
        def __reduce__(self):
            return (print, ("pwned",))
    bad = tmp_path / "bad.pkl"
    bad.write_bytes(pickle.dumps([Evil()]))
    with pytest.raises(pickle.UnpicklingError):
        T.load_itos(str(bad))


def test_generate_text_loop_feeds_tokens():
    itos = ["xxunk", "xxpad", "a", "b", ".", "c", "xxup"]
    stoi = T.make_stoi(itos)
    fed = []

    def step(tok):
        fed.append(tok)
        lg = torch.full((len(itos),), -1e4)
        lg[4 if len(fed) % 2 else 2] = 50.0
        lg[6] = 40.0
        return lg
    text = T.generate_text(step, lambda: None, itos, stoi, ["b"], n_words=4, generator=torch.Generator().manual_seed(0))
    assert fed[0] == stoi["b"]
    assert text == " b. A. A"
