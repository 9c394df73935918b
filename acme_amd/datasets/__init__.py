"""Datasets: the learner-side iterator over replay (acme/datasets)."""
from acme_amd.datasets.reverb import make_reverb_dataset, make_dataset  # noqa: F401
