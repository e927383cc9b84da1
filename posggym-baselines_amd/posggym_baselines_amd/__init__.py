"""posggym_baselines_amd — MI355X-native POMCP engine behind the
``posggym_baselines.planning`` API."""
__version__ = "0.1.0"
