"""Native WordPiece tokenizer (csrc/tokenizer.cpp) vs the python HF `tokenizers`
engine — the Rust engine tokenizers-cpp wraps (reference tokenizer.cpp:30-53) —
on the same tokenizer.json blob; plus bert_tokenize's framing
(reference bert.cpp:738-781).  CPU only: no model or GPU involved."""
import random

import pytest

import bertlib
from gguf_reader import GGUF

tokenizers = pytest.importorskip("tokenizers")

TEXTS = [
    "Québec",  # reference KAT string (examples/test_tokenizer.cpp:70)
    "syömme \t  täällä    tänään",  # reference KAT string
    "I'm going to the store to buy 3 apples and a banana! You're welcome to come along if you'd like.",
    "\"5 2 + 3 * 4 -\"; int stack[1000], top = -1; int calculate(int a, int b, char operator) { return a; }",
    "naïve café résumé ÅNGSTRÖM Ærøskøbing",
    "中文字符 and 日本語 and 한국어",
    "ba ce di fo gu babacedi bace ##x [CLS] [SEP] [UNK]",
    "x" * 101,
    "x" * 100,
    "tab\there\nline\r\ncr zero​width soft­hyphen",
    "İstanbul ΣΊΣΥΦΟΣ Ǆemal",
    "a.b,c;d!e?f(g)h[i]j{k}l<m>n@o#p$q%r^s&t*u_v-w+x=y~z`",
    "",
    "   ",
    "emoji 🙂 and math ∑ ∫ √",
]


@pytest.fixture(scope="module")
def tok_json(model_dir):
    import os
    p = os.path.join(model_dir, "tok_minilm_f16_l1.gguf")
    if not os.path.exists(p):
        bertlib.synth_model(p, "minilm", "f16", n_layer=1)
    return GGUF(p).kv["blob.tokenizer.json"]


def test_encode_matches_hf_tokenizers(tok_json):
    ref = tokenizers.Tokenizer.from_str(tok_json)
    for t in TEXTS:
        want = ref.encode(t, add_special_tokens=False).ids
        assert bertlib.tokenize_json(tok_json, t, n_max=4096) == want, t


def test_encode_random_strings(tok_json):
    ref = tokenizers.Tokenizer.from_str(tok_json)
    rng = random.Random(1234)
    alphabet = list("abcdefghijklmnopqrstuvwxyzABCDEFG  .,!?'\"-()0123456789") + list("éèüöäßçñåøæœ中日한ΣЖ")
    for _ in range(300):
        t = "".join(rng.choice(alphabet) for _ in range(rng.randint(0, 80)))
        assert bertlib.tokenize_json(tok_json, t, n_max=4096) == ref.encode(t, add_special_tokens=False).ids, t


def test_truncation_from_json(tok_json):
    # synthetic tokenizer.json truncates content to n_max_tokens - 2 (510)
    ref = tokenizers.Tokenizer.from_str(tok_json)
    t = " ".join(["ba"] * 700)
    ids = bertlib.tokenize_json(tok_json, t, n_max=4096)
    assert ids == ref.encode(t, add_special_tokens=False).ids
    assert len(ids) == 510


def test_bert_tokenize_framing(tok_json):
    # [CLS] + ids + [SEP]; truncation keeps [SEP] in the last slot (bert.cpp:772-779)
    ids = bertlib.tokenize_json(tok_json, "ba ce di fo gu", frame=False)
    framed = bertlib.tokenize_json(tok_json, "ba ce di fo gu", n_max=512, frame=True)
    assert framed == [101] + ids + [102]
    short = bertlib.tokenize_json(tok_json, "ba ce di fo gu", n_max=4, frame=True)
    assert short == [101] + ids[:2] + [102]
    assert bertlib.tokenize_json(tok_json, "", n_max=8, frame=True) == [101, 102]
