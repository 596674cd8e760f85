"""gmr — MI355X-native (gfx950) hot path of GenMMRec's DiffMM / DiffRec / VBPR.

The package mirrors the reference module API (GeneralRecommender models, Trainer /
DiffMMTrainer, get_model/get_trainer, Config, quick_start) and runs every hot op through
the hand-written HIP kernels of libgmr_hip.so (include/gmr.h).
"""
__version__ = "0.1.0"
