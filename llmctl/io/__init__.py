"""IO: synthetic / memmap token datasets, sampling, sharded async checkpoints."""
