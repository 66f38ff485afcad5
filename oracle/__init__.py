"""ORACLE — test infrastructure only.

CPU NumPy restatement of the HiFi-GAN V1 vocoder and FastSpeech2-Conformer acoustic
model, pinned against golden vectors from transformers 5.15.0 (tests/golden/).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import it;
the product package gonova_tts_amd never does.
"""
