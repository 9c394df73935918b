"""Environment wrappers needed by the drop-in agents."""
from acme_amd.wrappers.observation_action_reward import OAR, ObservationActionRewardWrapper  # noqa
