"""Golden token ids for the fixed-shape text tokenizer (run in the build container, where the reference
is readable; the fixture is committed, the reference is not read at test time).

Loads the reference's own `dataset/dataset_utils/tokenizer.py` and `text_transform_builder.py` by path.
`ftfy` is not installed in this image: a stand-in module whose `fix_text` returns its argument is put in
sys.modules before the load (ftfy leaves ASCII text unchanged, so the ASCII cases are the reference's
exact ids; the one non-ASCII caption is NFC-stable and quote-free, where ftfy is the identity as well).

    python tests/golden/make_token_golden.py [/root/reference]
"""
import importlib.util
import json
import os
import sys
import types

ref_root = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
utils = os.path.join(ref_root, "dataset", "dataset_utils")
sys.modules["ftfy"] = types.SimpleNamespace(fix_text=lambda t: t)
pkg = types.ModuleType("ref_dataset_utils")
pkg.__path__ = [utils]
sys.modules["ref_dataset_utils"] = pkg
for name in ("tokenizer", "text_transform_builder"):
    spec = importlib.util.spec_from_file_location(f"ref_dataset_utils.{name}", os.path.join(utils, f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
tok_mod = sys.modules["ref_dataset_utils.tokenizer"]
tt_mod = sys.modules["ref_dataset_utils.text_transform_builder"]

CAPTIONS = [
    "a brown wooden chair next to the table.",
    "There's a white door on the left wall; it's closed.",
    "TWO   monitors\ton the desk &amp; a keyboard",
    "3 pillows, 12 books and 1 lamp!!!",
    "",
    "they'll've we're I'm you'd",
    "a toilet-paper-holder (white) near the sink?",
    "<|startoftext|> special tokens <|endoftext|> inside",
    "a cafe table and a café chair",
    "the sofa is in front of the television and the coffee table " * 20,
    "kitchen cabinets above the counter, refrigerator to the right of the stove",
    "bookshelf",
]
tok = tok_mod.SimpleTokenizer()
out = {"encode": [{"text": t, "ids": tok.encode(t)} for t in CAPTIONS]}
cases = []
for max_len, crop, texts in ((120, 10, CAPTIONS), (77, 10, CAPTIONS[:3]), (16, 4, CAPTIONS[8:])):
    ids = tt_mod.text_transform(max_len, crop)(texts)
    cases.append({"max_seq_len": max_len, "cropped_texts": crop, "texts": texts, "ids": ids.tolist()})
out["text_transform"] = cases
out["specials"] = {"sot": tok.encoder["<|startoftext|>"], "eot": tok.encoder["<|endoftext|>"],
                   "vocab": len(tok.encoder)}
here = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(here, "tokens.json"), "w") as f:
    json.dump(out, f)
print("wrote tokens.json", out["specials"], [len(e["ids"]) for e in out["encode"]])
