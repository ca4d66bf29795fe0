"""``python -m llmctl`` == the ``llmctl`` console script."""

from llmctl.cli.main import app

if __name__ == "__main__":
    app(prog_name="llmctl")
