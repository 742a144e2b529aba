"""pyconsensus_amd -- MI355X-native Oracle.consensus() (PCA path) behind the pyconsensus API."""
__version__ = "0.1.0"
