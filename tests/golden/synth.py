"""Re-export of the seeded synthetic inputs / config used to generate and check fixtures."""
from rdeic_amd.config import CONFIG  # noqa: F401
from rdeic_amd.synthetic import sampler_noise, synth_context, synth_image  # noqa: F401
