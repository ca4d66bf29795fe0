"""Communications: RCCL collectives, DP overlap engine, PP p2p, xGMI topology."""
