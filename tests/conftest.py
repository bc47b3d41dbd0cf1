import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def pytest_report_header(config):
    """Name the build under test: the same library_sha16 that bench.py's JSON
    line and profiles/*_profile_summary.json carry, so a test record and a bench
    record can be matched to one library file."""
    from subproc_amd import _lib

    try:
        sha = _lib.library_sha16()
    except OSError:
        sha = "missing"
    return f"subproc_amd library_sha16={sha} ({os.path.relpath(_lib.LIB_PATH, ROOT)})"


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    # repeated at the end of the run, where a record that keeps only the tail sees it
    terminalreporter.write_line(pytest_report_header(config))
