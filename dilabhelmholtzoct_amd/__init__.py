"""dilabhelmholtzoct_amd — MI355X-native (gfx950 HIP) implementation of the OCT-SAM training-step
hot path of philippendres/DILabHelmholtzOCT (octsam/models/training_utils.py:41-69)."""
__version__ = "0.1.0"
