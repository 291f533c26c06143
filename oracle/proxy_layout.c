/* ORACLE (test infrastructure only): prints the proxy message layout of the
 * reference's own src/include/proxy/proxy.h (compiled where /root/reference
 * lies, oracle/Makefile `ref`), against which include/apus_gpu.h's
 * APUS_REC_* constants are checked (tests/test_records.py). */
#include <stddef.h>
#include <stdio.h>

#include "proxy/proxy.h"

int main(void)
{
    printf("{\"header\": %zu, \"connect\": %zu, \"close\": %zu, \"send\": %zu, \"send_data\": %zu, "
           "\"action\": %zu, \"connection_id\": %zu, \"CONNECT\": %d, \"SEND\": %d, \"CLOSE\": %d}\n",
           sizeof(proxy_msg_header), sizeof(proxy_connect_msg), sizeof(proxy_close_msg), sizeof(proxy_send_msg),
           offsetof(proxy_send_msg, data), offsetof(proxy_msg_header, action),
           offsetof(proxy_msg_header, connection_id), CONNECT, SEND, CLOSE);
    return 0;
}
