"""Fixed-shape text tokenization for the text branch of config 5.

Restates `dataset/dataset_utils/text_transform_builder.py:33-76` (`text_transform(max_seq_len,
cropped_texts)`: keep the first `cropped_texts` captions, wrap each in start/end-of-text tokens, pad with
0 to `max_seq_len`, truncate long captions to `max_seq_len` with end-of-text in the last slot) over the
CLIP byte-level BPE of `dataset/dataset_utils/tokenizer.py:87-146` (the published CLIP tokenizer:
GPT-2's byte->unicode table, lower-cased text split by CLIP's regex, greedy lowest-rank pair merges,
49152 - 256 - 2 merges, vocabulary = 256 bytes, 256 bytes + '</w>', the merges, then
<|startoftext|> 49406 and <|endoftext|> 49407).

The merges list is the reference's own data file (`bpe_simple_vocab_16e6.txt.gz`, the CLIP vocabulary),
shipped here as package data (wsss3d/data/).  The reference cleans text with `ftfy.fix_text`, which is
not installed in this image: `_fix_text` is the identity on ASCII (ftfy's fixes only touch non-ASCII
text, and line breaks, which the whitespace clean-up removes anyway) and otherwise applies ftfy's
default NFC normalisation and quote uncurling only -- token ids of non-ASCII captions are therefore
parity-unpinned.  Token ids of ASCII captions are pinned against the reference tokenizer by
tests/golden/tokens.json (tests/golden/make_token_golden.py).

TextTransformer (wsss3d/text.py) picks each caption's feature at `text.argmax(-1)`, i.e. the
end-of-text token, the largest id.
"""
from __future__ import annotations

import gzip
import html
import os
import unicodedata
from functools import lru_cache

import regex
import torch

VOCAB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "bpe_simple_vocab_16e6.txt.gz")
N_MERGES = 49152 - 256 - 2
SOT, EOT = "<|startoftext|>", "<|endoftext|>"
# CLIP's pre-tokenisation pattern (tokenizer.py:99-101): special tokens, English contractions, runs of
# letters, single digits, runs of other non-space characters
_SPLIT = regex.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|"""
                       r"""[^\s\p{L}\p{N}]+""", regex.IGNORECASE)
_QUOTES = str.maketrans({"‘": "'", "’": "'", "‚": "'", "‛": "'",
                         "“": '"', "”": '"', "„": '"', "‟": '"'})


@lru_cache()
def byte_alphabet():
    """GPT-2's reversible byte -> printable character table: printable Latin-1 bytes map to themselves,
    the other 68 bytes to 256, 257, ... in byte order."""
    keep = [b for b in range(256) if (33 <= b <= 126) or (161 <= b <= 172) or (174 <= b <= 255)]
    table, extra = {}, 0
    for b in range(256):
        if b in keep:
            table[b] = chr(b)
        else:
            table[b] = chr(256 + extra)
            extra += 1
    # the vocabulary lists the bytes in this order: the kept ones first, then the remapped ones
    return {b: table[b] for b in keep + [b for b in range(256) if b not in keep]}


def _fix_text(text):
    if text.isascii():
        return text
    return unicodedata.normalize("NFC", text).translate(_QUOTES)


def clean(text):
    """tokenizer.py basic_clean + whitespace_clean + lower-casing (encode)."""
    text = html.unescape(html.unescape(_fix_text(text))).strip()
    return regex.sub(r"\s+", " ", text).strip().lower()


class SimpleTokenizer:
    """CLIP byte-level BPE (encode / decode) over the reference's merges file."""

    def __init__(self, bpe_path: str = VOCAB_PATH):
        with gzip.open(bpe_path) as f:
            lines = f.read().decode("utf-8").split("\n")
        merges = [tuple(line.split()) for line in lines[1:N_MERGES + 1]]
        self.byte_encoder = byte_alphabet()
        self.byte_decoder = {c: b for b, c in self.byte_encoder.items()}
        symbols = list(self.byte_encoder.values())
        vocab = symbols + [s + "</w>" for s in symbols] + ["".join(m) for m in merges] + [SOT, EOT]
        self.encoder = {tok: i for i, tok in enumerate(vocab)}
        self.decoder = {i: tok for tok, i in self.encoder.items()}
        self.bpe_ranks = {m: r for r, m in enumerate(merges)}
        self._memo = {SOT: (SOT,), EOT: (EOT,)}

    def bpe(self, token: str):
        """Symbols of one pre-token after BPE: start from its characters (the last one marked '</w>'),
        then repeatedly merge every occurrence (left to right, non-overlapping) of the adjacent pair with
        the lowest merge rank until no adjacent pair has a rank."""
        hit = self._memo.get(token)
        if hit is not None:
            return hit
        word = list(token[:-1]) + [token[-1] + "</w>"]
        ranks = self.bpe_ranks
        while len(word) > 1:
            best, best_rank = None, None
            for pair in zip(word, word[1:]):
                r = ranks.get(pair)
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = pair, r
            if best is None:
                break
            a, b = best
            merged, i = [], 0
            while i < len(word):
                if i + 1 < len(word) and word[i] == a and word[i + 1] == b:
                    merged.append(a + b)
                    i += 2
                else:
                    merged.append(word[i])
                    i += 1
            word = merged
        out = tuple(word)
        self._memo[token] = out
        return out

    def encode(self, text: str):
        ids = []
        for piece in _SPLIT.findall(clean(text)):
            mapped = "".join(self.byte_encoder[b] for b in piece.encode("utf-8"))
            ids.extend(self.encoder[s] for s in self.bpe(mapped))
        return ids

    def decode(self, ids):
        text = "".join(self.decoder[int(i)] for i in ids)
        raw = bytearray(self.byte_decoder[c] for c in text)
        return raw.decode("utf-8", errors="replace").replace("</w>", " ")


@lru_cache()
def default_tokenizer():
    return SimpleTokenizer()


class Tokenize:
    """text_transform_builder.py Tokenize: captions -> (n, max_seq_len) int64, 0-padded; a caption longer
    than max_seq_len is cut to max_seq_len with end-of-text in the last slot (truncate=True) or raises."""

    def __init__(self, tokenizer, max_seq_len: int, truncate: bool = True):
        self.tokenizer, self.max_seq_len, self.truncate = tokenizer, int(max_seq_len), truncate

    def __call__(self, texts):
        single = isinstance(texts, str)
        if single:
            texts = [texts]
        sot, eot = self.tokenizer.encoder[SOT], self.tokenizer.encoder[EOT]
        out = torch.zeros(len(texts), self.max_seq_len, dtype=torch.long)
        for row, text in enumerate(texts):
            ids = [sot] + self.tokenizer.encode(text) + [eot]
            if len(ids) > self.max_seq_len:
                if not self.truncate:
                    raise RuntimeError(f"Input {text} is too long for context length {self.max_seq_len}")
                ids = ids[:self.max_seq_len - 1] + [eot]
            out[row, :len(ids)] = torch.tensor(ids, dtype=torch.long)
        return out[0] if single else out


class WordSplitTokenizeWrapper:
    """text_transform_builder.py WordSplitTokenizeWrapper: tokenize the first `cropped_num` captions."""

    def __init__(self, tokenize, cropped_num: int):
        self.tokenize, self.num_texts = tokenize, int(cropped_num)

    def __call__(self, texts):
        return self.tokenize(texts[:self.num_texts])


def text_transform(max_seq_len: int, cropped_texts: int):
    """text_transform_builder.py:33-35 (the configs use max_seq_len 120, cropped_texts 10,
    config/3DUNetWithText_scannet_default.yaml:14-15)."""
    return WordSplitTokenizeWrapper(Tokenize(default_tokenizer(), max_seq_len=max_seq_len), cropped_texts)
