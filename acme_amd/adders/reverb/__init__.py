"""Replay adders — drop-in for `acme.adders.reverb` (same class names and arguments).

They write through the Reverb writer surface (`client.writer(...)`, `append`,
`create_item`, `close`); `acme_amd.replay.Client` implements it on top of the GPU
replay table, so the adders run unchanged against device-resident replay.
"""

from acme_amd.adders.reverb._common import (DEFAULT_PRIORITY_TABLE, PriorityFn,  # noqa: F401
                                            PriorityFnInput, PriorityFnMapping, ReverbAdder,
                                            Step, calculate_priorities, final_step_like,
                                            zeros_like)
from acme_amd.adders.reverb._items import (EpisodeAdder, NStepTransitionAdder,  # noqa: F401
                                           SequenceAdder)
