"""Worker plugins — drop-ins for the reference's workers/*.py."""
