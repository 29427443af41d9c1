"""ORACLE — test infrastructure only.

CPU restatement of the reference (ShreyasBhaktharam/RDEIC) hot path, used by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg as the *checker*; the product
(rdeic_amd) never imports this package.

Parity status: the NN graph restatement (oracle/model_ref.py) is pinned against golden
fixtures produced by the reference's own modules (tests/golden/, tests/golden/make_golden.py).
The entropy coders (oracle/coders_ref.py) restate compressai 1.2.4 / torchac 0.9.3, which are
not present in the reference tree: they are pinned by known-answer vectors (the torchac uniform
hyper-latent code) and round-trip properties, and are otherwise "parity unpinned" (SURVEY.md §8c).
"""
