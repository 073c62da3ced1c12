"""MI355X-native frequency-domain EMRI waveform generator (FD mode-sum hot path)."""
