// TEST DOUBLE -- MgenBaseEvent::GetStringFromProtocol and the DrecEvent getters LogDrecEvent
// reads (reference include/mgenEvent.h), for the protolib-branch build of compat_shapes.
#pragma once
#include <stdio.h>

#include "protokit.h"
#include "mgenGlobals.h"

class MgenBaseEvent {
 public:
  static const char* GetStringFromProtocol(Protocol p) {
    switch (p) {
      case UDP: return "UDP";
      case TCP: return "TCP";
      case SINK: return "SINK";
      default: return "UNKNOWN";
    }
  }
};

class DrecEvent : public MgenBaseEvent {
 public:
  Protocol GetProtocol() const { return protocol; }
  const ProtoAddress& GetGroupAddress() const { return group_addr; }
  const ProtoAddress& GetSourceAddress() const { return source_addr; }
  const char* GetInterface() const { return iface[0] ? iface : NULL; }
  void SetProtocol(Protocol p) { protocol = p; }
  void SetGroupAddress(const ProtoAddress& a) { group_addr = a; }
  void SetSourceAddress(const ProtoAddress& a) { source_addr = a; }
  void SetInterface(const char* name) { snprintf(iface, sizeof(iface), "%s", name ? name : ""); }

 private:
  Protocol protocol = INVALID_PROTOCOL;
  ProtoAddress group_addr, source_addr;
  char iface[64] = {0};
};
