// Native stress test of the shm request/response protocol (csrc/host/shm_core.h), built with
// -fsanitize=thread (or address) by tests/test_shm_channel.py.  One server thread, N client threads,
// each client on its own slot; every response must echo its request's payload checksum.
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "../../applestar_amd/csrc/host/shm_core.h"

using namespace as_host;

int main(int argc, char** argv) {
  const int n_clients = argc > 1 ? std::atoi(argv[1]) : 4;
  const int n_req = argc > 2 ? std::atoi(argv[2]) : 500;
  const std::string name = "/applestar_stress_" + std::to_string(getpid());
  ServerCore server(name, n_clients, 8192);
  std::vector<int> bad(n_clients, 0);
  std::vector<std::thread> clients;
  for (int c = 0; c < n_clients; ++c) {
    clients.emplace_back([&, c] {
      ClientCore cl(name, c, 7 + c);
      std::vector<uint8_t> buf(64 + c);
      for (int r = 0; r < n_req; ++r) {
        uint32_t sum = 0;
        for (size_t k = 0; k < buf.size(); ++k) {
          buf[k] = static_cast<uint8_t>(r * 31 + k * 7 + c);
          sum += buf[k];
        }
        if (cl.request(buf.data(), buf.size(), 20000) != Wait::kOk) { bad[c]++; continue; }
        uint32_t got = 0;
        std::memcpy(&got, cl.response_data(), sizeof(got));
        if (cl.response_len() != sizeof(got) || got != sum) bad[c]++;
      }
    });
  }
  long served = 0;
  const long total = static_cast<long>(n_clients) * n_req;
  while (served < total) {
    for (uint32_t s : server.wait(1000)) {
      const uint8_t* p = reinterpret_cast<const uint8_t*>(server.request_data(s));
      uint32_t sum = 0;
      for (size_t k = 0; k < server.request_len(s); ++k) sum += p[k];
      if (server.tag(s) != 7 + s) sum ^= 0xdeadbeef;
      server.respond(s, &sum, sizeof(sum));
      ++served;
    }
  }
  for (auto& t : clients) t.join();
  int errors = 0;
  for (int b : bad) errors += b;
  std::printf("%s served=%ld errors=%d\n", errors ? "FAIL" : "OK", served, errors);
  return errors ? 1 : 0;
}
