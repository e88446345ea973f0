"""The native GET /inference route's detokenizer table (serve/native_http.py lm_route_table, read by
csrc/http.cpp try_lm): for any token sequence the text it assembles, JSON-escaped, equals the
Flask route's json.dumps of the Detokenizer's text (serve/text.py) -- including capitalisation
after ".", "!" and newlines, NO_SPACE words whose capitalised form is not in NO_SPACE ("n't"
-> "N't"), quotes, backslashes and non-ASCII words."""
import json
import random

from hipzap.serve.native_http import lm_route_table, render_with_table
from hipzap.serve.server import synthetic_vocab
from hipzap.serve.text import Detokenizer


def _flask_text(itos, ids):
    det = Detokenizer()
    det.add_prompt("")
    for t in ids:
        det.add(itos[t])
    return json.dumps({"response": {"text": det.text}})


def test_table_render_equals_the_flask_body():
    itos = synthetic_vocab(300) + ["n't", "'ll", "\\n", "Ünïcødé", "quo\"te", "back\\slash", " ", "é", "!",
                                   "HTTP", "http", "ǆemal", "straße", "\t", "😀x"]
    blob, flags = lm_route_table(itos)
    rng = random.Random(0)
    specials = [i for i, w in enumerate(itos) if not w.isalpha()]
    for _ in range(300):
        ids = [rng.choice(specials) if rng.random() < 0.4 else rng.randrange(len(itos)) for _ in range(rng.randint(1, 60))]
        body = '{"response": {"text": "' + render_with_table(blob, flags, ids) + '"}}'
        assert body == _flask_text(itos, ids), ids
        assert json.loads(body)  # valid JSON
