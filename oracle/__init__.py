"""CPU oracle for the GenMMRec DiffMM/DiffRec/VBPR hot path — TEST INFRASTRUCTURE ONLY.

This package is a CPU restatement of the reference algorithm, used as the
checker for the HIP path.  It is imported only by tests/, by
__graft_entry__.smoke() and by bench.py's ``cpu_baseline`` leg.  The product
path (generative-multimodal-recommendation_amd/gmr) never imports it and fails
loudly when the HIP library is missing.

Parity status: PINNED.  Every function here is checked against golden vectors
produced by importing the reference itself (tests/golden/make_golden.py ->
tests/golden/*.npz, checked by tests/test_oracle_golden.py).

Modules
  graph_ref   integer/byte work: CSR builds of the normalised adjacencies (numpy, fp64 math)
  model_ref   floating-point work: DiffMM / DiffRec / VBPR restated in torch-CPU fp32
  eval_ref    top-K selection and Recall/NDCG/Precision/MAP (numpy)
"""
