"""opentsdb_amd: MI355X engine for OpenTSDB query-time aggregation (libtsdbhip)."""
