"""Parallelism strategies: TP/SP (tensor_parallel), PP (pipeline), ZeRO-1/2/3 (zero),
DP (llmctl.comms.overlap), process-group construction (groups)."""
