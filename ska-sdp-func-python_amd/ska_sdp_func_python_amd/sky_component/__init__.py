"""Sky-component helpers used by the sky-model drivers."""
from .operations import apply_beam_to_skycomponent  # noqa: F401
