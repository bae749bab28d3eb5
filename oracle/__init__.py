"""CPU oracle package (test infrastructure only; see srt_oracle.h)."""
