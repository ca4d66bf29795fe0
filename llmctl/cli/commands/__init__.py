"""Subcommand modules (one Typer app each)."""
