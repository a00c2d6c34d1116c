"""Text front end (magpie.cpp:124-495) and sentence splitter (4439-4480): the C++
implementation in libmagpie_hip.so against the pure-Python restatement in
oracle/tokenizer_ref.py, on the synthetic GGUF's vocabulary/dictionary. The
known-answer cases pin the restatement to the reference's rules as written
(number words with "and", year pairs, ordinal compounds, currency, percent,
negatives, punctuation tokens without a following space, letter fallback)."""
import random

import pytest

from gguf_kv import read_kv
from oracle import tokenizer_ref as ref


@pytest.fixture(scope="module")
def tok_pair(small_model):
    import magpie_amd as ma
    kv = read_kv(small_model)
    vocab = kv["magpie.tokenizer.vocab"].decode("utf-8")
    dct = kv["magpie.tokenizer.dict"].decode("utf-8")
    return ma.Tokenizer(small_model), ref.load(vocab, dct, space=kv["magpie.tokenizer.space"])


@pytest.mark.parametrize("text,words", [
    ("$1", "one dollar"), ("$50", "fifty dollars"), ("2024", "twenty twenty four"), ("1900", "nineteen hundred"),
    ("2001", "two thousand one"), ("2100", "two thousand one hundred"), ("21st", "twenty first"),
    ("101st", "one hundred and first"), ("3rd", "third"), ("40th", "fortieth"), ("13th", "thirteenth"),
    ("-5", "minus five"), ("-0", "zero"), ("15%", "fifteen percent"), ("-2%", "minus two percent"),
    ("12345", "twelve thousand three hundred and forty five"),
    ("1234567", "one million two hundred and thirty four thousand five hundred and sixty seven"),
    ("7000000000", "seven billion"), ("1000000000000", "1000000000000"), ("0th", "zeroth"),
])
def test_normalisation_known_answers(text, words):
    assert ref.normalize_text(text) == words


def test_tokenizer_matches_restatement(tok_pair):
    cpp, py = tok_pair
    fixed = ["Hello, world!", "Hello world", "I paid $50 on the 21st of May 2024; 15% more.", "Joy and voice",
             "-3 degrees", "THE FIRST VOICE", "a.b,c", "twenty", "   spaced   out   ", "", "tabs\tinside words",
             "multi\nline", "Ünïcödé wörds", "4th 22nd 103rd 1999 1000 2099 2100 9999"]
    rng = random.Random(0)
    alphabet = list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJ0123456789  ,.!?:;$%-'") + ["hello", "world", "the ",
                                                                                      "voice", "joy", "é", "日"]
    for _ in range(300):
        fixed.append("".join(rng.choice(alphabet) for _ in range(rng.randint(1, 40))))
    for t in fixed:
        assert cpp(t) == ref.tokenize(py, t), repr(t)


def test_tokenizer_structure(tok_pair):
    cpp, _ = tok_pair
    ids = cpp("Hello, world!")
    assert ids[0] == 2378 and ids[-1] == 2379
    assert 93 in ids and ids[-2] != 93  # spaces between words, none before EOS


def test_split_sentences_matches_restatement():
    import magpie_amd as ma
    cases = ["Hello world. How are you? Fine!", "No boundary here", "Decimal 3.5 stays. End.", "Trailing   ",
             "  Lead. \n Next!\tLast?", "Wait...what? Yes.", "", "   ", "a.b. c", "One.\nTwo"]
    rng = random.Random(1)
    for _ in range(200):
        cases.append("".join(rng.choice("ab .!?\n\t") for _ in range(rng.randint(0, 30))))
    for t in cases:
        assert ma.split_sentences(t) == ref.split_sentences(t), repr(t)
