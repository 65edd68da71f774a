"""ORACLE — TEST INFRASTRUCTURE ONLY.

A CPU restatement of keras-geometric's MessagePassing.propagate() hot path as
the reference executes it: Keras-3 ops lowered to PyTorch ATen CPU kernels
(KERAS_BACKEND=torch, reference .env:1).  It exists to CHECK the kgx HIP
engine and to time the reference's CPU path; it is never the thing measured
or shipped.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import it.  The product package (keras-geometric_amd/) never imports
it and has no CPU fallback.

Provenance / pinning
--------------------
* The reference (src/keras_geometric, snapshot 2025-06-20) cannot be imported
  here: `import keras_geometric` fails with ModuleNotFoundError: keras (an
  ordinary error, not a permission denial).  Keras is pinned
  only as keras>=3.0 (reference pyproject.toml:33), so the Keras-torch
  lowering of each keras.ops call is restated in oracle/keras_torch.py from
  Keras 3.x's torch backend (keras/src/backend/torch/{math,numpy,nn}.py,
  ≈3.10) — names and semantics cited per function.
* The restatement is pinned by the reference's own known-answer tests
  (tests/test_message_passing.py:54-179, tests/unit/test_error_handling.py,
  tests/test_graphsage_conv.py:465-514) — see tests/test_oracle_pins.py — and
  by cross-checks against plain sequential numpy loops (oracle/sequential.py).
* PyTorch-Geometric comparisons in the reference tests need torch_geometric,
  which is not installed.  The algorithms they compare against (PyG >= 2.6.1,
  reference pyproject.toml:51: gcn_norm + GCNConv, GATv2Conv, GINConv) are
  restated in float64 numpy in oracle/pyg_restated.py, and
  tests/test_oracle_pyg_pins.py holds the oracle to them at those tests'
  tolerances -- this pins the GCN normalisation (utils/main.py:20-33) and the
  GATv2 segment softmax (gatv2_conv.py:268-311), which no reference-held
  vector covers.
"""

ORACLE_IS_TEST_INFRASTRUCTURE = True
