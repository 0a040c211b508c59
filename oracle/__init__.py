"""Oracle package: CPU restatement of the reference path (test infrastructure only)."""
