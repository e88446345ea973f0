"""Vocabulary I/O, the reference's sampling rule and detokenizer (GET /inference parity).

Behaviour reproduced from /root/reference/main.py:40-81 (read, not copied):
  * prompt words are fed one token at a time; unknown words map to id 0 (main.py:54-57);
  * every generation step draws 10 ids WITHOUT replacement with probability proportional to
    exp(logits) (``torch.multinomial(res[-1].exp(), 10)``, main.py:61) and keeps the first id
    that is neither 0 nor one of {xxup, xxfld, xxrep}; if none qualifies, the first draw
    (main.py:47, 63-68);
  * detokenizer: no space before the tokens of ``NO_SPACE`` (main.py:45, 75-78); a word is
    capitalised when the previous emitted word is '.', '!' or '\\n' (main.py:46, 73);
  * the returned text starts with ' ' + each prompt word (main.py:57).
Sampling here is Gumbel-top-k over the logits — the same Plackett-Luce distribution as
multinomial-without-replacement on exp(logits), but computed in log space (the reference's
``exp`` overflows fp32 for logits > ~88). Parity is therefore distributional, not bitwise
(torch's CPU RNG stream cannot be reproduced); tests check it statistically.
"""
from __future__ import annotations

import io
import pickle

# (annotations only -- ``typing`` and ``json`` are imported where used: the torch-free LM cold-start
# child imports this module on its critical path)

NO_SPACE = ["'s", "'ll", ",", "?", ".", "'t", "'m", "n't", "!", "'", "'ve", ";", "http", ":", "/", "\\"]
CAPITALIZE_AFTER = [".", "!", "\n"]
EXCLUDE_TOKENS = ["xxup", "xxfld", "xxrep"]
NUM_DRAWS = 10


class _NoGlobalsUnpickler(pickle.Unpickler):
    """Unpickler that refuses every global: plain lists/strings load, code never runs."""

    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from a vocabulary file")


def load_itos(path: str) -> list[str]:
    """Load a vocabulary (``.itos.pkl`` list[str] as the reference stores it, or JSON)."""
    with open(path, "rb") as f:
        data = f.read()
    if path.endswith(".json"):
        import json
        itos = json.loads(data.decode("utf-8"))
    else:
        itos = _NoGlobalsUnpickler(io.BytesIO(data)).load()
    if not isinstance(itos, (list, tuple)) or not all(isinstance(s, str) for s in itos):
        raise ValueError("vocabulary must be a list of strings")
    return list(itos)


def save_itos(itos: Sequence[str], path: str) -> None:
    if path.endswith(".json"):
        with open(path, "w") as f:
            import json
            json.dump(list(itos), f)
    else:
        with open(path, "wb") as f:
            pickle.dump(list(itos), f)


def make_stoi(itos: Sequence[str]) -> dict[str, int]:
    # main.py:93 builds {w: i} by enumeration: later duplicates win
    return {w: i for i, w in enumerate(itos)}


def gumbel_topk(logits: torch.Tensor, k: int, generator: torch.Generator | None = None) -> torch.Tensor:
    """k draws without replacement, P ∝ exp(logits) (Plackett-Luce), in log space."""
    import torch
    lg = logits.float().reshape(-1)
    u = torch.rand(lg.shape, generator=generator, device=lg.device).clamp_(1e-20, 1.0)
    g = -torch.log(-torch.log(u))
    return torch.topk(lg + g, min(k, lg.numel())).indices


def select_token(draws: Sequence[int], exclude: set[int]) -> int:
    """main.py:63-68: first draw that is not 0 and not excluded, else the first draw."""
    for r in draws:
        if r != 0 and r not in exclude:
            return int(r)
    return int(draws[0])


class Detokenizer:
    def __init__(self):
        self.text = ""
        self.last = None

    def add_prompt(self, word: str):
        self.text += " " + word

    def add(self, word: str) -> str:
        if self.last in CAPITALIZE_AFTER:
            word = word.capitalize()
        self.text = self.text + word if word in NO_SPACE else self.text + " " + word
        self.last = word
        return word


def generate_text(step: Callable[[int], torch.Tensor], reset: Callable[[], None], itos: Sequence[str],
                  stoi: dict, prompt_words: Sequence[str], n_words: int = 200,
                  generator: torch.Generator | None = None,
                  sampler: Callable[[torch.Tensor, int], Sequence[int]] | None = None) -> str:
    """The reference's generation loop (main.py:40-81) over any ``step(token) -> logits``.

    ``sampler(logits, k)`` may be a device-side sampler returning the k draws; default is
    host Gumbel-top-k.
    """
    exclude = {stoi[w] for w in EXCLUDE_TOKENS if w in stoi}
    reset()
    det = Detokenizer()
    logits = None
    for w in prompt_words:
        logits = step(stoi.get(w, 0))
        det.add_prompt(w)
    if logits is None:
        raise ValueError("need at least one prompt word (the reference uses [''])")
    for _ in range(n_words):
        draws = sampler(logits, NUM_DRAWS) if sampler else gumbel_topk(logits, NUM_DRAWS, generator).tolist()
        tok = select_token(list(draws), exclude)
        logits = step(tok)
        det.add(itos[tok])
    return det.text
