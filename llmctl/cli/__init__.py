"""llmctl command-line interface."""
