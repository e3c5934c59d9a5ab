"""Peer-to-peer wire protocol and headers-first sync."""
