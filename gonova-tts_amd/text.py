"""Text front end: sentence segmentation (reference behaviour) and a deterministic
character tokenizer for the 78-symbol acoustic-model vocabulary.

`split_into_sentences` reproduces the reference's offline path exactly
(`services/tts/core/synthesizer.py:48-99`, regex fallback `:73-76` — spaCy is not
installed and its model download at `:36-40` needs the network), including its
comma/semicolon re-chunking at `max_chars` and the `", "` re-join.

The published FastSpeech2-Conformer tokenizer needs `g2p_en` (not installed;
SURVEY.md §8f rank 4), so tokens are a fixed character map: 0 = <blank>/pad,
1 = <unk>, 2.. = characters, 77 = <sos/eos> appended at the end (espnet's
convention of ending every sequence with the sos/eos symbol).
"""
from __future__ import annotations

import re
from typing import List

import numpy as np

PAD_ID = 0
UNK_ID = 1
EOS_ID = 77
_CHARS = " abcdefghijklmnopqrstuvwxyz0123456789'.,!?-;:\"()&/%$@#+=*_~<>[]{}|\\^`"
CHAR_TO_ID = {c: i + 2 for i, c in enumerate(_CHARS)}
assert max(CHAR_TO_ID.values()) < EOS_ID


def split_into_sentences(text: str, max_chars: int = 150) -> List[str]:
    """Reference `split_into_sentences` (synthesizer.py:48-99), regex path."""
    text = text.strip()
    if not text:
        return []
    sentences = re.split(r'(?<=[.!?])\s+(?=[A-Z])', text)
    sentences = [s.strip() for s in sentences if s.strip()]
    result = []
    for sentence in sentences:
        if len(sentence) <= max_chars:
            result.append(sentence)
        else:
            parts = re.split(r'[,;]\s+', sentence)
            current = ""
            for part in parts:
                if not current:
                    current = part
                elif len(current) + len(part) + 2 <= max_chars:
                    current += ", " + part
                else:
                    result.append(current)
                    current = part
            if current:
                result.append(current)
    return result


def tokenize(text: str, add_eos: bool = True) -> np.ndarray:
    """Deterministic char -> id map (lower-cased, whitespace collapsed)."""
    s = " ".join(text.lower().split())
    ids = [CHAR_TO_ID.get(c, UNK_ID) for c in s]
    if add_eos:
        ids.append(EOS_ID)
    if not ids:
        ids = [EOS_ID]
    return np.asarray(ids, dtype=np.int32)


def tokenize_batch(texts: List[str]):
    """-> (tokens int32 [B, N] zero-padded, lengths int32 [B])."""
    seqs = [tokenize(t) for t in texts]
    n = max(len(s) for s in seqs)
    out = np.zeros((len(seqs), n), np.int32)
    for i, s in enumerate(seqs):
        out[i, : len(s)] = s
    return out, np.asarray([len(s) for s in seqs], np.int32)
