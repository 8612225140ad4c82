"""Drop-in entry points: `python -m scripts.<name>` from robust-object-detection_amd/, as in the reference."""
