"""AWD-LSTM: checkpoint compatibility with the reference module, W_hh quirk, stateful API."""
import importlib.util
import os
import sys

import pytest
import torch

from hipzap.models.awd_lstm import get_language_model

REF = "/root/reference/pytorch_models/awd_lstm.py"


def _ref_module():
    if not os.path.exists(REF):
        pytest.skip("reference not mounted")
    spec = importlib.util.spec_from_file_location("ref_awd_lstm", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


KW = dict(vocab_sz=120, emb_sz=40, n_hid=48, n_layers=3, pad_token=1, tie_weights=True, bias=True, qrnn=False)


def test_state_dict_keys_match_reference():
    ref = _ref_module().get_language_model(**KW)
    ours = get_language_model(**KW)
    assert set(ref.state_dict()) == set(ours.state_dict())
    for k, v in ref.state_dict().items():
        assert ours.state_dict()[k].shape == v.shape, k


def test_forward_matches_reference_eval():
    ref = _ref_module().get_language_model(**KW)
    ours = get_language_model(**KW)
    sd = ref.state_dict()
    ours.load_state_dict(sd)
    ref.eval(); ours.eval()
    ref.reset(); ours.reset()
    torch.manual_seed(0)
    for step in range(5):
        x = torch.randint(0, 120, (3, 2))
        with torch.no_grad():
            a, ra, oa = ref(x)
            b, rb, ob = ours(x)
        assert a.shape == b.shape == (6, 120)
        assert torch.allclose(a, b, atol=1e-5), step
        assert len(rb) == len(ob) == 3


def test_whh_quirk_module_weight_wins():
    ours = get_language_model(**KW)
    sd = ours.state_dict()
    sd = {k: v.clone() for k, v in sd.items()}
    for l in range(3):
        sd[f"0.rnns.{l}.weight_hh_l0_raw"].zero_()
        sd[f"0.rnns.{l}.module.weight_hh_l0"].fill_(0.5)
    ours.load_state_dict(sd)
    assert torch.all(ours[0].rnns[0].module.weight_hh_l0 == 0.5)
    assert torch.all(ours[0].rnns[0].weight_hh_l0_raw == 0.5)


def test_tied_decoder_and_hidden_reset_on_batch_change():
    m = get_language_model(**KW).eval()
    assert m[1].decoder.weight.data_ptr() == m[0].encoder.weight.data_ptr()
    m(torch.zeros(1, 1, dtype=torch.long))
    h1 = m[0].hidden[0][0].clone()
    assert h1.abs().sum() > 0
    m(torch.zeros(1, 3, dtype=torch.long))
    assert m[0].bs == 3 and m[0].hidden[0][0].shape[1] == 3


def test_qrnn_unsupported():
    with pytest.raises(NotImplementedError):
        get_language_model(**dict(KW, qrnn=True))


def test_bidirectional_core_matches_reference():
    """bidir=True (reference awd_lstm.py:57,69-70,95): same keys and shapes, same eval forward."""
    kw = dict(KW, bidir=True)
    ref = _ref_module().get_language_model(**kw)
    ours = get_language_model(**kw)
    assert set(ref.state_dict()) == set(ours.state_dict())
    sd = ref.state_dict()
    ours.load_state_dict(sd)
    ref.eval(); ours.eval()
    ref.reset(); ours.reset()
    x = torch.randint(0, KW["vocab_sz"], (7, 3))
    with torch.no_grad():
        a = ref(x)[0]
        b = ours(x)[0]
    assert torch.allclose(a, b, atol=1e-5)
    assert ours[0].hidden[0][0].shape == (2, 3, KW["n_hid"] // 2)


def test_bidirectional_checkpoint_refused_by_gpu_packer():
    from hipzap.engine.lm import pack_awd_lstm
    sd = get_language_model(**dict(KW, bidir=True)).state_dict()
    with pytest.raises(ValueError, match="bidirectional"):
        pack_awd_lstm(sd, "cpu")
